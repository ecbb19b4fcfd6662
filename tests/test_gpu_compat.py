"""Drop-in trainer / scanner surface end to end on the GPU (synthetic faces on disk)."""
import json
import os
import pickle

import numpy as np
import pytest

from oracle import eigenface_oracle as orc

pytestmark = pytest.mark.gpu


def _person_dir(root, person, n, seed):
    from PIL import Image
    d = os.path.join(root, "faces", "lock_version", person)
    os.makedirs(d)
    x, _ = orc.synth_faces(n, 64, r=32, seed=seed)
    faces = []
    for i, row in enumerate(x):
        fn = f"face_{i:04d}.png"
        Image.fromarray(row.reshape(64, 64), mode="L").save(os.path.join(d, fn))
        # Windows-style path as in the committed JSONs: resolved via image_filename
        faces.append({"face_id": i, "image_path": f"faces\\lock_version\\{person}\\{fn}", "image_filename": fn,
                      "width": 64, "height": 64})
    json.dump({"faces": faces}, open(os.path.join(d, f"{person}_faces_detection.json"), "w"))
    return x


def test_train_v4_cli_and_pickle(tmp_path):
    from eigenface.cli import train_v4
    from eigenface.compat import FaceTrainer, recognize_face_all_models
    from eigenface import recognize_face_with_model
    xa = _person_dir(str(tmp_path), "alice", 120, 1)
    xb = _person_dir(str(tmp_path), "bob", 90, 2)
    assert train_v4("alice", str(tmp_path)) == 0
    assert train_v4("bob", str(tmp_path)) == 0
    base = tmp_path / "faces" / "lock_version"
    for p in ("alice", "bob"):
        assert (base / p / "face_model.pkl").exists()
        assert (base / p / f"{p}_model_info.json").exists()
        assert (base / p / f"{p}_eigenface_01.jpg").exists() and (base / p / f"{p}_mean_face.jpg").exists()
    md = pickle.load(open(base / "alice" / "face_model.pkl", "rb"))  # written by this package
    assert set(md) >= {"pca", "scaler", "face_features", "face_labels", "face_info", "person_id_map",
                       "n_components", "mean_face", "eigenfaces", "face_shape", "training_date"}
    # the pickled sklearn objects reproduce the oracle's sklearn path (train-v4.py:131-134)
    ref = orc.train_pca_model(xa, 50)
    f_ref = orc.sklearn_transform(xa[:10], ref["scaler"], ref["pca"])
    f_pk = md["pca"].transform(md["scaler"].transform(xa[:10].astype(np.float64)))
    scale = np.abs(f_ref).max()
    # components agree up to sign only where the spectrum has gaps: compare projections' norms
    np.testing.assert_allclose(np.linalg.norm(f_pk, axis=1), np.linalg.norm(f_ref, axis=1), rtol=1e-6)
    np.testing.assert_allclose(md["pca"].explained_variance_, ref["pca"]["explained_variance_"], rtol=1e-8)
    np.testing.assert_allclose(md["face_features"][:, :10], ref["face_features"][:, :10], atol=1e-6 * scale)
    # reference-style recognition on the loaded dict (scan-template-v4.py:270-287)
    pid, name, sim = recognize_face_with_model(f_pk[3], md, 0.8)
    assert (pid, name) == (0, "alice") and sim > 0.999
    # multi-model best (scan-template-v4.py:289-319)
    models = {p: {"model_data": pickle.load(open(base / p / "face_model.pkl", "rb"))} for p in ("alice", "bob")}
    assert recognize_face_all_models(xa[5].reshape(64, 64), models, 0.8)[1] == "alice"
    assert recognize_face_all_models(xb[7].reshape(64, 64), models, 0.8)[1] == "bob"
    tr = FaceTrainer()
    assert tr.load_model(str(base / "bob" / "face_model.pkl")) and tr.person_id_map == {"bob": 0}


def test_train_manual_cli(tmp_path):
    from PIL import Image
    from eigenface.cli import train_manual
    d = tmp_path / "faces_in"
    d.mkdir()
    x, _ = orc.synth_faces(150, 40, r=24, seed=8)
    for i, row in enumerate(x):
        Image.fromarray(row.reshape(40, 40), mode="L").save(d / f"img_{i:03d}.png")
    assert train_manual(str(d), "carol", str(tmp_path / "models"), "light", 20) == 0
    meta = json.load(open(tmp_path / "models" / "carol_light_model_info.json"))
    _, _, _, lam = orc.manual_pca(x, 20)
    np.testing.assert_allclose(meta["explained_variance_ratio"], orc.manual_model_info_evr(lam), rtol=1e-9)
    md = pickle.load(open(tmp_path / "models" / "carol_light_pca_model.pkl", "rb"))
    assert md["eigenfaces"].shape == (1600, 20) and md["training_filenames"][0] == "img_000.png"
    from eigenface import recognize_face
    name, sim, ok = recognize_face(x[11].astype(np.float64), md, 0.7)
    assert name == "carol" and ok and sim > 0.9999


def test_read_faces_gpu_ingest_matches_oracle(tmp_path):
    """compat.read_faces: host decode + one GPU grey/resize launch == the OpenCV-rule
    restatement (oracle/image_oracle.py); unreadable files are skipped."""
    from PIL import Image
    from eigenface.compat import read_face, read_faces
    from oracle import image_oracle as io
    rng = np.random.default_rng(9)
    paths, ref = [], []
    for i, shp in enumerate([(100, 100, 3), (224, 230, 3), (37, 53), (128, 128, 3)]):
        a = rng.integers(0, 256, shp, dtype=np.uint8)
        p = str(tmp_path / f"f{i}.png")
        Image.fromarray(a).save(p)
        paths.append(p)
        bgr = a[..., ::-1] if a.ndim == 3 else a
        ref.append(io.preprocess(bgr, (64, 64)))
    paths.insert(2, str(tmp_path / "missing.png"))
    rows, keep = read_faces(paths)
    assert keep == [0, 1, 3, 4]
    np.testing.assert_array_equal(rows, np.stack(ref))
    np.testing.assert_array_equal(read_face(paths[0]).ravel(), ref[0])
    assert read_face(paths[2]) is None


def test_engine_owner_tokens_interleaved_models():
    """Two EigenfacePCA instances and the drop-in functions share one engine per device:
    each must re-upload its model / gallery when another caller replaced it (owner
    tokens), never silently use someone else's."""
    from eigenface import EigenfacePCA, recognize_face_with_model
    xa, _ = orc.synth_faces(300, 32, r=24, seed=41)
    xb, _ = orc.synth_faces(300, 32, r=24, seed=42)
    a = EigenfacePCA(12, standardize=True).fit(xa)
    b = EigenfacePCA(12, standardize=True).fit(xb)
    fa = a.transform(xa[:5])
    fb = b.transform(xb[:5])
    ia, _ = a.recognize(xa[:5])
    ib, _ = b.recognize(xb[:5])
    for _ in range(2):  # interleave: each call must see its own model and gallery
        np.testing.assert_allclose(a.transform(xa[:5]), fa, rtol=1e-6, atol=1e-6)
        np.testing.assert_array_equal(b.recognize(xb[:5])[0], ib)
        np.testing.assert_allclose(b.transform(xb[:5]), fb, rtol=1e-6, atol=1e-6)
        np.testing.assert_array_equal(a.recognize(xa[:5])[0], ia)
    np.testing.assert_array_equal(ia, np.arange(5))
    # a drop-in recognise with another gallery in between
    g = np.random.default_rng(3).standard_normal((50, 12))
    md = {"face_features": g, "face_labels": np.arange(50), "person_id_map": {f"p{i}": i for i in range(50)}}
    pid, _, _ = recognize_face_with_model(g[7], md, threshold=0.5)
    assert pid == 7
    np.testing.assert_array_equal(a.recognize(xa[:5])[0], ia)
    g[7] = -g[7]  # in-place edit of the same array: the digest forces a re-upload
    pid, _, _ = recognize_face_with_model(g[7], md, threshold=0.5)
    assert pid == 7
