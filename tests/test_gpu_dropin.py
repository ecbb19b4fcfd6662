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
