"""The reference-named drop-in entry files run as the reference's callers run them:
``python train-v4.py --person P`` (run_pipeline.py:234, subprocess.run with check=True at
:41) and ``python train-v5.py`` from a checkout root, then the scanner's model discovery
(scan-template-v4.py:17-74) and batched recognition over the written models."""
import json
import os
import pickle
import subprocess
import sys

import numpy as np
import pytest

from conftest import PKG
from oracle import eigenface_oracle as orc
from oracle import image_oracle as io

pytestmark = pytest.mark.gpu

DROPIN = os.path.join(PKG, "dropin")


def _write_person(root, person, n, seed, with_json=True, size=(72, 80)):
    """JPEG crops of synthetic faces (BGR, size h x w) under faces/lock_version/person, a
    detection JSON with cwd-relative image paths as detection-v4.py writes them
    (detection-v4.py:64-88).  Returns the rows the trainers must see: libjpeg decode ->
    cvtColor(BGR2GRAY) -> resize(64, 64) by the OpenCV-rule restatement."""
    from PIL import Image
    from eigenface.compat import decode_image
    d = os.path.join(root, "faces", "lock_version", person)
    os.makedirs(d)
    x, _ = orc.synth_faces(n, 64, r=32, seed=seed)
    rng = np.random.default_rng(seed)
    faces, rows = [], []
    for i, row in enumerate(x):
        g = np.asarray(Image.fromarray(row.reshape(64, 64), mode="L").resize((size[1], size[0])), np.uint8)
        bgr = np.stack([g, np.clip(g.astype(int) + rng.integers(-6, 7), 0, 255), g], -1).astype(np.uint8)
        fn = f"face_{i:06d}_frame_{10 * i:06d}.jpg"
        Image.fromarray(bgr[..., ::-1]).save(os.path.join(d, fn), quality=95)
        rows.append(io.preprocess(decode_image(os.path.join(d, fn)), (64, 64)))
        faces.append({"face_id": i, "frame_number": 10 * i, "x": 0, "y": 0, "width": size[1], "height": size[0],
                      "image_path": os.path.join("faces", "lock_version", person, fn), "image_filename": fn})
    if with_json:
        json.dump({"faces": faces}, open(os.path.join(d, f"{person}_faces_detection.json"), "w"))
    return np.stack(rows)


def _run(script, root, *args):
    env = dict(os.environ)
    return subprocess.run([sys.executable, os.path.join(DROPIN, script), *args], cwd=root, env=env,
                          capture_output=True, text=True, timeout=240)


def test_train_v4_dropin_subprocess_and_scanner(tmp_path, monkeypatch):
    root = str(tmp_path)
    xa = _write_person(root, "alice", 110, 1)
    xb = _write_person(root, "bob", 95, 2)
    for p in ("alice", "bob"):
        r = _run("train-v4.py", root, "--person", p)
        assert r.returncode == 0, r.stderr[-2000:]
        assert "Training completed successfully!" in r.stdout
    # a missing person prints the reference's error and still exits 0 (train-v4.py:281-284)
    r = _run("train-v4.py", root, "--person", "nobody")
    assert r.returncode == 0 and "not found" in r.stdout
    base = tmp_path / "faces" / "lock_version"
    for p in ("alice", "bob"):
        info = json.load(open(base / p / f"{p}_model_info.json"))
        assert info["person_name"] == p and info["n_components"] == 50 and info["eigenfaces_saved"] == 10
    # the fit saw exactly the decoded/grey/resized rows: sklearn-path oracle on them
    md = pickle.load(open(base / "alice" / "face_model.pkl", "rb"))
    ref = orc.train_pca_model(xa, 50)
    np.testing.assert_allclose(md["pca"].explained_variance_, ref["pca"]["explained_variance_"], rtol=1e-8)
    np.testing.assert_allclose(md["mean_face"], xa.mean(axis=0), rtol=1e-13)
    # scanner model discovery (scan-template-v4.py:17-74): cwd-relative template paths
    from eigenface.compat import load_all_models, recognize_faces_all_models
    monkeypatch.chdir(root)
    models = load_all_models(".")
    assert list(models) == ["alice", "bob"]
    for p in ("alice", "bob"):
        t = models[p]["template_images"]
        assert len(t) == 5 and t[0]["image"].shape == (72, 80) and (t[0]["width"], t[0]["height"]) == (80, 72)
        assert models[p]["detection_data"]["faces"][0]["face_id"] == 0
    # batched best-over-models recognition of crops (scan-template-v4.py:289-319)
    crops = [xa[3].reshape(64, 64), xb[7].reshape(64, 64), xa[50].reshape(64, 64)]
    res = recognize_faces_all_models(crops, models, 0.8)
    assert [r[1] for r in res] == ["alice", "bob", "alice"]
    assert all(r[2] > 0.99 for r in res)


def test_train_v5_dropin_full_rank_vs_oracle(tmp_path):
    """train-v5.py: k = face count (full rank).  The first n-1 components / eigenvalues
    match the oracle's sklearn 'full' fit at k = n; the last component is the null
    direction (eigenvalue ~0): a unit vector orthogonal to the others, training features
    ~0 on it (sklearn's is LAPACK's arbitrary null vector: unpinned)."""
    root = str(tmp_path)
    xc = _write_person(root, "carol", 70, 5, with_json=False)  # JSON synthesised by train-v5
    xd = _write_person(root, "dave", 64, 6)
    r = _run("train-v5.py", root)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "Successful trainings: 2" in r.stdout
    base = tmp_path / "faces" / "lock_version"
    assert (base / "carol" / "carol_faces_detection.json").exists()
    det = json.load(open(base / "carol" / "carol_faces_detection.json"))
    assert det["total_faces_detected"] == 70 and det["faces"][3]["frame_number"] == 30
    for p, x in (("carol", xc), ("dave", xd)):
        n = len(x)
        info = json.load(open(base / p / "multi_person_model_info.json"))
        assert info["n_components"] == n and info["total_persons"] == 1 and info["person_id_map"] == {p: 0}
        assert (base / p / "multi_person_eigenface_10.jpg").exists()
        md = pickle.load(open(base / p / "face_model.pkl", "rb"))
        assert md["n_components"] == n and md["face_features"].shape == (n, n)
        # carol's rows follow its synthesised JSON = sorted file names = generation order
        ref = orc.train_pca_model(x, n)
        lam, lam_ref = md["pca"].explained_variance_, ref["pca"]["explained_variance_"]
        np.testing.assert_allclose(lam[:n - 1], lam_ref[:n - 1], rtol=1e-8)
        assert abs(lam[-1]) < 1e-9 * lam[0] and abs(lam_ref[-1]) < 1e-9 * lam_ref[0]
        C = md["pca"].components_
        np.testing.assert_allclose(C @ C.T, np.eye(n), atol=1e-9)  # incl. the null component
        gap = np.ones(n - 1, bool)
        rel = np.abs(np.diff(lam_ref[:n - 1])) / lam_ref[0]
        gap[:-1] &= rel > 1e-6
        gap[1:] &= rel > 1e-6
        np.testing.assert_allclose(C[:n - 1][gap], ref["pca"]["components_"][:n - 1][gap], atol=1e-7)
        F = md["face_features"]
        assert np.abs(F[:, -1]).max() < 1e-6 * np.abs(F).max()


def test_train_v5_601_faces_recognised_at_full_rank(tmp_path, monkeypatch):
    """The reference's own faces/lock_version/shun holds 601 crops, so train-v5.py
    (n_components = face count, train-v5.py:539-545) writes a k = 601 model.  Recognition
    against it (scan-template-v4.py:265-287, batched as recognize_faces_all_models) runs the
    k > 512 projection and cosine search and returns the oracle's first-argmax identities."""
    root = str(tmp_path)
    n = 601
    xs = _write_person(root, "shun", n, 21, size=(64, 64))
    r = _run("train-v5.py", root)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "Successful trainings: 1" in r.stdout
    base = tmp_path / "faces" / "lock_version" / "shun"
    md = pickle.load(open(base / "face_model.pkl", "rb"))
    assert md["n_components"] == n and md["face_features"].shape == (n, n)
    from eigenface.compat import load_all_models, recognize_faces_all_models
    monkeypatch.chdir(root)
    models = load_all_models(".")
    assert list(models) == ["shun"]
    # probes: 40 training crops (their own rows must win) + 24 unseen faces of the same kind
    unseen, _ = orc.synth_faces(24, 64, r=32, seed=99)
    pick = np.arange(0, n, 15)[:40]
    probes = np.concatenate([xs[pick], unseen])
    res = recognize_faces_all_models([p.reshape(64, 64) for p in probes], models, 0.8)
    assert len(res) == len(probes)
    # oracle: sklearn transform of the pickled estimators in fp64, cosine first-argmax vs the
    # pickled training features, threshold >= (scan-template-v4.py:265-287)
    sc, pca = md["scaler"], md["pca"]
    f = orc.sklearn_transform(probes, (sc.mean_, sc.var_, sc.scale_),
                              {"components_": pca.components_, "mean_": pca.mean_})
    s = orc.cosine_scores(f, md["face_features"])
    ref_idx = np.argmax(s, axis=1)
    srt = np.sort(s, axis=1)
    clear = (srt[:, -1] - srt[:, -2]) > 1e-5
    assert clear[:40].all()
    for j, (pid, name, conf) in enumerate(res):
        assert abs(conf - s[j, ref_idx[j]]) < 1e-5
        if not clear[j]:
            continue
        if s[j, ref_idx[j]] >= 0.8:
            assert pid == md["face_labels"][ref_idx[j]] and name == "shun"
        else:
            assert pid == -1 and name == "shun"  # below threshold: the model's person name
    # the training crops are recognised as themselves (labels are all shun's id)
    assert all(res[j][1] == "shun" and res[j][2] > 0.999 for j in range(40))
    # and the engine's own argmax row for them is the crop's own training row
    from eigenface.compat import extract_faces_features
    from eigenface.pca import _gallery_engine
    feats = extract_faces_features(probes[:40], md)
    idx, _ = _gallery_engine(md["face_features"], 0).search(feats.astype(np.float32), "cosine")
    np.testing.assert_array_equal(idx, ref_idx[:40])
    np.testing.assert_array_equal(idx, pick)
