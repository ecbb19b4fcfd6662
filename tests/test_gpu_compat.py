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
    assert train_v4("alice", str(tmp_path)) is True
    assert train_v4("bob", str(tmp_path)) is True
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


def test_read_faces_and_grey_decode_jpeg_on_gpu(tmp_path):
    """JPEG files go through the GPU decoder (ef_jpeg_ingest / ef_jpeg_decode): the rows
    equal libjpeg-turbo's pixels (Pillow) through the resize oracle; a progressive JPEG and
    a PNG take the host decoder inside the same call."""
    import jpeg_cases as J
    from eigenface.compat import read_faces, read_gray_images
    from oracle import image_oracle as io
    paths, blobs = [], []
    for i, (h, w, sub) in enumerate([(120, 96, 2), (61, 77, 0), (200, 150, 1)]):
        b = J.encode(J.smooth_image(h, w, 3, i), quality=95, subsampling=sub)
        blobs.append(b)
    blobs.append(J.encode(J.smooth_image(90, 90, 3, 7), quality=80, progressive=True))
    for i, b in enumerate(blobs):
        p = tmp_path / f"face_{i}.jpg"
        p.write_bytes(b)
        paths.append(str(p))
    from PIL import Image
    png = J.smooth_image(50, 70, 3, 9)
    Image.fromarray(png).save(tmp_path / "face_png.png")
    paths.append(str(tmp_path / "face_png.png"))
    rows, keep = read_faces(paths)
    assert keep == [0, 1, 2, 3, 4]
    for i in range(4):
        np.testing.assert_array_equal(rows[i], io.preprocess(J.decode_ref(blobs[i], "bgr"), (64, 64)))
    np.testing.assert_array_equal(rows[4], io.preprocess(png[..., ::-1], (64, 64)))
    grey = read_gray_images(paths[:4])
    for i in range(4):
        np.testing.assert_array_equal(grey[i], J.decode_ref(blobs[i], "gray"))


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


def _describe(v):
    if isinstance(v, np.ndarray):
        return {"type": "ndarray", "dtype": str(v.dtype), "shape": list(v.shape),
                "f_contiguous": bool(v.flags.f_contiguous), "c_contiguous": bool(v.flags.c_contiguous)}
    return {"type": type(v).__name__}


def test_config1_synthetic_manual_path_vs_reference(tmp_path):
    """BASELINE config 1 without photographs: an exact-integer synthetic stand-in of
    faces/Light_version (229 faces, 100 x 100) through cli.train_manual (useless/train.py
    train_single_model: sorted files -> manual_pca k=50 -> models/*_pca_model.pkl +
    *_model_info.json) and recognize_face, against the reference's own manual_pca,
    save_pca_model and recognize_face outputs (tests/golden/make_goldens.py c1)."""
    from PIL import Image
    from conftest import golden
    from eigenface import recognize_face, recognize_faces
    from eigenface.cli import train_manual
    g = golden("c1_synth.npz")
    X = orc.int_synth_faces(int(g["n"]), int(g["side"]), r=int(g["r"]), seed=int(g["seed"]))
    d = tmp_path / "Light_version"
    d.mkdir()
    side = int(g["side"])
    for i, row in enumerate(X):
        Image.fromarray(row.reshape(side, side), mode="L").save(d / f"img_{i:03d}.png")
    assert train_manual(str(d), "synth", str(tmp_path / "models"), "light", int(g["k"])) == 0
    md = pickle.load(open(tmp_path / "models" / "synth_light_pca_model.pkl", "rb"))  # written by this package
    info = json.load(open(tmp_path / "models" / "synth_light_model_info.json"))
    layout = json.loads(str(g["layout"]))
    assert {k: _describe(v) for k, v in md.items()} == layout["pkl"]
    assert sorted(info) == layout["info_keys"]
    assert md["training_filenames"][:2] == ["img_000.png", "img_001.png"] and md["version"] == "light"
    np.testing.assert_allclose(md["eigenvalues"], g["eigenvalues"], rtol=1e-9)
    np.testing.assert_allclose(info["explained_variance_ratio"], g["evr_json"], rtol=1e-9)
    np.testing.assert_allclose(md["mean_face"].sum(), float(g["mean_sum"]), rtol=1e-14)
    R = np.random.default_rng([5]).integers(0, 2, size=(X.shape[1], 8)).astype(np.float64) * 2.0 - 1.0
    er = md["eigenfaces"].T @ R
    s = np.sign((er * g["eigenfaces_R"]).sum(axis=1))
    np.testing.assert_allclose(er * s[:, None], g["eigenfaces_R"], atol=1e-4)
    proj = md["projected_data"] * s[None, :]
    np.testing.assert_allclose(proj, g["projected"], atol=1e-6 * np.abs(g["projected"]).max())
    # recognise (useless/scan.py:100-132) one by one and batched
    sims = []
    for p, want_sim, want_ok in zip(g["probes"], g["sim"], g["recognized"]):
        name, sim, ok = recognize_face(p.astype(np.float64), md, 0.7)
        assert name == "synth" and ok == bool(want_ok)
        sims.append(sim)
    # fp32 projection: |f32 - f| <= 2e-6 * sum|p - mu||w| per component (the K6 bound,
    # tests/test_gpu_project.py); the cosine moves by at most 2 |df| / |f| — large only for
    # the mean-face probe, whose projection is nearly all cancellation
    P = g["probes"].astype(np.float64) - md["mean_face"]
    f = P @ md["eigenfaces"]
    df = 2e-6 * (np.abs(P) @ np.abs(md["eigenfaces"]))
    tol = 2 * np.linalg.norm(df, axis=1) / np.linalg.norm(f, axis=1) + 1e-6
    assert np.all(np.abs(np.array(sims) - g["sim"]) <= tol)
    batch = recognize_faces(g["probes"], md, 0.7)
    np.testing.assert_allclose([b[1] for b in batch], sims, atol=1e-6)


def test_dual_model_recognition_matches_reference_rule():
    """recognize_face_dual_model (useless/scan.py:134-166): OR of the two models'
    decisions, max similarity, the dark model's name on ties; against the oracle's
    single-model recognise per model."""
    from eigenface import manual_pca, recognize_face_dual_model
    xd = orc.int_synth_faces(120, 24, r=40, seed=11)
    xl = orc.int_synth_faces(140, 24, r=40, seed=12)
    models = []
    for nm, x in (("dark", xd), ("light", xl)):
        e, m, p, lam = manual_pca(x, 20)
        models.append({"eigenfaces": e, "mean_face": m, "projected_data": p, "person_name": f"joe_{nm}"})
    rng = np.random.default_rng(1)
    probes = np.concatenate([xd[:3], xl[:3], rng.integers(0, 256, (2, xd.shape[1]))]).astype(np.uint8)
    for v in probes:
        got = recognize_face_dual_model(v, models[0], models[1], 0.7)
        rd = orc.recognize_face_manual(v, models[0], 0.7)
        rl = orc.recognize_face_manual(v, models[1], 0.7)
        assert got[2] == (rd[2] or rl[2])
        assert got[0] == (rd[0] if rd[1] >= rl[1] else rl[0]) or abs(rd[1] - rl[1]) < 1e-6
        np.testing.assert_allclose(got[3:], [rd[1], rl[1]], atol=2e-6)
        np.testing.assert_allclose(got[1], max(rd[1], rl[1]), atol=2e-6)


def test_gallery_cache_recognize(tmp_path):
    """EigenfacePCA.save_gallery / set_gallery(path): the memory-mapped cache gives the same
    identities as the in-memory gallery."""
    import numpy as np
    from eigenface import EigenfacePCA
    from oracle import eigenface_oracle as orc
    x, _ = orc.synth_faces(300, 32, r=24, seed=3)
    m = EigenfacePCA(20).fit(x)
    idx0, s0 = m.recognize(x[:50], "cosine")
    p = m.save_gallery(tmp_path / "g.npy")
    m2 = EigenfacePCA(20).fit(x)
    m2.set_gallery(p)
    idx1, s1 = m2.recognize(x[:50], "cosine")
    np.testing.assert_array_equal(idx1, idx0)
    np.testing.assert_array_equal(s1, s0)


def test_model_without_pca_key_is_skipped_like_the_reference(tmp_path, capsys):
    """a face_model.pkl keyed 'pca_model' instead of 'pca' — the layout of
    the reference's own faces/lock_version/Joseph_Lai/face_model.pkl (SURVEY Appendix A:
    float32 arrays, mean_face = pca.mean_; rebuilt here synthetically, the reference's
    pickle is not read) — raises KeyError('pca') at scan-template-v4.py:266; the per-model
    try prints "Error recognizing with model <name>: 'pca'" and skips the model (:312-314).
    Alone it yields (-1, 'unknown', 0.0) for every face; beside a well-formed model it
    changes nothing."""
    from eigenface.cli import train_v4
    from eigenface.compat import load_all_models, recognize_face_all_models, recognize_faces_all_models
    xa = _person_dir(str(tmp_path), "alice", 120, 1)
    assert train_v4("alice", str(tmp_path)) is True
    base = tmp_path / "faces" / "lock_version"
    good = pickle.load(open(base / "alice" / "face_model.pkl", "rb"))  # written by this package
    bad = {k: v for k, v in good.items() if k != "pca"}
    bad["pca_model"] = good["pca"]
    for key in ("face_features", "eigenfaces"):
        bad[key] = np.asarray(good[key], dtype=np.float32)
    bad["mean_face"] = np.asarray(good["pca"].mean_, dtype=np.float32)
    bad["person_id_map"] = {"joseph": 0}
    jdir = tmp_path / "solo" / "faces" / "lock_version" / "joseph"
    jdir.mkdir(parents=True)
    pickle.dump(bad, open(jdir / "face_model.pkl", "wb"))
    faces = [xa[i].reshape(64, 64) for i in (0, 5, 17, 33)]

    solo = load_all_models(str(tmp_path / "solo"))
    assert list(solo) == ["joseph"]
    capsys.readouterr()
    assert recognize_faces_all_models(faces, solo, 0.8) == [(-1, "unknown", 0.0)] * len(faces)
    assert "Error recognizing with model joseph: 'pca'" in capsys.readouterr().out
    assert recognize_face_all_models(faces[0], solo, 0.8) == (-1, "unknown", 0.0)

    only_good = {"alice": {"model_data": good}}
    want = recognize_faces_all_models(faces, only_good, 0.8)
    assert [w[1] for w in want] == ["alice"] * len(faces)
    both = {"alice": {"model_data": good}, "joseph": {"model_data": bad}}
    capsys.readouterr()
    assert recognize_faces_all_models(faces, both, 0.8) == want
    assert "Error recognizing with model joseph: 'pca'" in capsys.readouterr().out
    both_rev = {"joseph": {"model_data": bad}, "alice": {"model_data": good}}
    assert recognize_faces_all_models(faces, both_rev, 0.8) == want


def test_resident_check_identity_mode():
    """set_resident_check('identity') skips the per-call digest; an in-place edit
    then needs invalidate_uploads (documented contract), after which the edit is seen."""
    from eigenface import invalidate_uploads, recognize_face_with_model, set_resident_check
    g = np.random.default_rng(4).standard_normal((64, 10))
    md = {"face_features": g, "face_labels": np.arange(64), "person_id_map": {f"p{i}": i for i in range(64)}}
    set_resident_check("identity")
    try:
        assert recognize_face_with_model(g[9], md, threshold=0.5)[0] == 9
        assert recognize_face_with_model(g[9], md, threshold=0.5)[0] == 9
        g[9] = -g[9]
        invalidate_uploads()
        assert recognize_face_with_model(g[9], md, threshold=0.5)[0] == 9
    finally:
        set_resident_check("digest")
    g[3] = -g[3]  # digest mode again: the edit is caught without invalidation
    assert recognize_face_with_model(g[3], md, threshold=0.5)[0] == 3
