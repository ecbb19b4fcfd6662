"""Format writers and sklearn object population (no GPU): layouts of
useless/train.py:130-192 and train-v4.py:199-228, checked with oracle arrays."""
import json
import os
import pickle
from types import SimpleNamespace

import numpy as np

from conftest import golden
from oracle import eigenface_oracle as orc


def test_save_pca_model_layout(tmp_path):
    from eigenface.compat import save_pca_model
    x, _ = orc.synth_faces(40, 16, r=8, seed=4)
    eig, mean, proj, lam = orc.manual_pca(x, 12)
    names = [f"f{i:03d}.jpg" for i in range(40)]
    path = save_pca_model(eig, mean, proj, lam, names, "P", str(tmp_path), "light")
    assert os.path.basename(path) == "P_light_pca_model.pkl"
    md = pickle.load(open(path, "rb"))  # our own file
    assert set(md) == {"eigenfaces", "mean_face", "projected_data", "eigenvalues", "training_filenames",
                       "person_name", "version", "training_timestamp", "n_components", "face_dimensions"}
    assert md["n_components"] == 12 and md["face_dimensions"] == 256
    meta = json.load(open(tmp_path / "P_light_model_info.json"))
    assert meta["model_file"] == "P_light_pca_model.pkl" and meta["n_training_images"] == 40
    assert meta["version"] == "light"
    np.testing.assert_allclose(meta["explained_variance_ratio"], orc.manual_model_info_evr(lam))
    save_pca_model(eig, mean, proj, lam, names, "Q", str(tmp_path))
    assert (tmp_path / "Q_pca_model.pkl").exists() and (tmp_path / "Q_model_info.json").exists()


def test_sklearn_objects_roundtrip_transform():
    """Populated sklearn StandardScaler/PCA reproduce the reference's transform
    (scan-template-v4.py:265-266) on the sklearn golden."""
    from eigenface.compat import sklearn_objects
    g = golden("sklearn_path.npz")
    r = orc.train_pca_model(g["X"], 16)
    p = r["pca"]
    fake = SimpleNamespace(
        standardize=True, n_features_in_=g["X"].shape[1], n_samples_=g["X"].shape[0], n_components=16,
        n_components_=16, scaler_mean_=r["scaler"][0], scaler_var_=r["scaler"][1], scaler_scale_=r["scaler"][2],
        mean_=p["mean_"], components_=p["components_"], explained_variance_=p["explained_variance_"],
        explained_variance_ratio_=p["explained_variance_ratio_"], singular_values_=p["singular_values_"],
        noise_variance_=p["noise_variance_"])
    scaler, pca = sklearn_objects(fake)
    scaler, pca = pickle.loads(pickle.dumps((scaler, pca)))
    f = pca.transform(scaler.transform(g["probes"].astype(np.float64)))
    np.testing.assert_allclose(f, g["probe_features"], rtol=1e-9, atol=1e-8)


def test_decode_image_is_bgr(tmp_path):
    """Host decode feeding the GPU ingest: BGR channel order like cv2.imread."""
    from PIL import Image
    from eigenface.compat import decode_image
    rgb = np.zeros((50, 40, 3), np.uint8)
    rgb[..., 0], rgb[..., 1], rgb[..., 2] = 200, 100, 50
    Image.fromarray(rgb).save(tmp_path / "a.png")
    g = decode_image(str(tmp_path / "a.png"))
    assert g.shape == (50, 40, 3) and tuple(g[0, 0]) == (50, 100, 200)
    Image.fromarray(rgb[..., 0]).save(tmp_path / "g.png")
    assert decode_image(str(tmp_path / "g.png")).shape == (50, 40)
    assert decode_image(str(tmp_path / "missing.png")) is None


def test_gallery_cache_roundtrip(tmp_path):
    """Raw .npy gallery-feature cache: float32, no pickle, memory-mapped load."""
    import numpy as np
    from eigenface import load_gallery_cache, save_gallery_cache
    g = np.random.default_rng(0).standard_normal((1000, 50))
    p = tmp_path / "gallery.npy"
    save_gallery_cache(p, g)
    a = load_gallery_cache(p)
    assert isinstance(a, np.memmap) and a.dtype == np.float32 and a.shape == (1000, 50)
    np.testing.assert_array_equal(a, g.astype(np.float32))
    np.save(tmp_path / "bad.npy", np.zeros(5))
    import pytest
    with pytest.raises(ValueError):
        load_gallery_cache(tmp_path / "bad.npy")


def test_upload_token_sees_any_inplace_edit():
    """The owner token of an uploaded gallery digests every byte: editing one row of a
    large gallery in place (re-enrolling a person) is seen, wherever the row is, so the
    next recognise call re-uploads instead of searching a stale device copy (the
    reference reads the array it is given on every call)."""
    from eigenface.pca import _ArrayToken
    rng = np.random.default_rng(0)
    g = rng.standard_normal((200_000, 32)).astype(np.float32)  # 25.6 MB
    tok = _ArrayToken(g)
    assert tok.matches(g)
    for row in (0, 1, 12_345, 99_999, 199_999):
        old = g[row].copy()
        g[row, 7] += 1.0
        assert not tok.matches(g), row
        g[row] = old
        assert tok.matches(g)
    assert not tok.matches(g.copy())  # another array with the same bytes is another owner
    import eigenface
    assert callable(eigenface.invalidate_uploads)
