"""The CPU oracle against the reference's own outputs (tests/golden, made by
tests/golden/make_goldens.py from the reference code) and the EVR the reference
committed in models/*_model_info.json."""
import numpy as np

from conftest import golden, local_golden
from oracle import eigenface_oracle as orc


def _sign_align(a, ref):
    s = np.sign((a * ref).sum(axis=0))
    s[s == 0] = 1
    return a * s


def test_light_manual_pca_matches_reference():
    g = local_golden("light_manual_pca.npz")
    eig, mean, proj, lam = orc.manual_pca(g["X"].astype(np.float64), 50)
    assert eig.shape == (10000, 50) and proj.shape == (229, 50)
    np.testing.assert_allclose(lam, g["eigenvalues"], rtol=1e-12)
    np.testing.assert_allclose(mean, g["mean_face"], rtol=0, atol=1e-12)
    e10 = _sign_align(eig[:, :10], g["eigenfaces_10"].astype(np.float64))
    np.testing.assert_allclose(e10, g["eigenfaces_10"], atol=1e-6)
    p = _sign_align(proj, g["projected"])
    np.testing.assert_allclose(p, g["projected"], rtol=1e-9, atol=1e-7)


def test_light_and_dark_evr_match_committed_model_info():
    g = golden("light_stats.npz")
    np.testing.assert_allclose(orc.manual_model_info_evr(g["eigenvalues"]), g["evr_json"], atol=1e-13)
    d = golden("dark_evr.npz")
    np.testing.assert_allclose(orc.manual_model_info_evr(d["eigenvalues"]), d["evr_json"], atol=1e-13)


def test_sklearn_path_matches_reference():
    g = golden("sklearn_path.npz")
    r = orc.train_pca_model(g["X"], 16)
    m, v, s = r["scaler"]
    np.testing.assert_allclose(m, g["scaler_mean"], rtol=1e-14)
    np.testing.assert_allclose(v, g["scaler_var"], rtol=1e-10)
    np.testing.assert_allclose(s, g["scaler_scale"], rtol=1e-10)
    p = r["pca"]
    np.testing.assert_allclose(p["components_"], g["components"], atol=1e-10)
    np.testing.assert_allclose(p["explained_variance_"], g["explained_variance"], rtol=1e-10)
    np.testing.assert_allclose(p["explained_variance_ratio_"], g["explained_variance_ratio"], rtol=1e-10)
    np.testing.assert_allclose(p["singular_values_"], g["singular_values"], rtol=1e-10)
    np.testing.assert_allclose(p["noise_variance_"], g["noise_variance"], rtol=1e-9)
    np.testing.assert_allclose(r["face_features"], g["face_features"], rtol=1e-9, atol=1e-8)
    np.testing.assert_allclose(r["mean_face"], g["mean_face"], rtol=1e-14)


def test_sklearn_probe_features_and_recognition():
    g = golden("sklearn_path.npz")
    r = orc.train_pca_model(g["X"], 16)
    f = orc.sklearn_transform(g["probes"], r["scaler"], r["pca"])
    np.testing.assert_allclose(f, g["probe_features"], rtol=1e-9, atol=1e-8)
    mu_f, w = orc.fold_projection(r["scaler"], r["pca"])
    np.testing.assert_allclose(orc.project(g["probes"], mu_f, w), g["probe_features"], rtol=1e-8, atol=1e-7)
    pid_map = {"alice": 0, "bob": 1, "carol": 2, "dave": 3, "erin": 4}
    for i, fv in enumerate(f):
        pid, _, sim = orc.recognize_face_with_model(fv, r["face_features"], g["labels"], pid_map, float(g["threshold"]))
        assert int(pid) == int(g["probe_person_id"][i])
        assert abs(sim - g["probe_similarity"][i]) < 1e-9


def test_tie_break_and_zero_norm():
    g = golden("ties.npz")
    idx, sim = orc.cosine_argmax(g["probes"], g["gallery"])
    np.testing.assert_array_equal(idx, g["idx"])
    np.testing.assert_allclose(sim, g["sim"], atol=1e-12)


def test_manual_scan_similarity():
    g = local_golden("manual_scan.npz")
    l = local_golden("light_manual_pca.npz")
    eig, mean, proj, _ = orc.manual_pca(l["X"], 50)
    model = {"eigenfaces": eig, "mean_face": mean, "projected_data": proj, "person_name": "Joseph_Lai"}
    for v, s, ok in zip(g["probes"], g["sim"], g["recognized"]):
        name, best, rec = orc.recognize_face_manual(v, model, 0.7)
        assert name == "Joseph_Lai"
        assert abs(best - s) < 1e-9 and rec == bool(ok)


def test_l2_argmin_lowest_index_on_ties():
    g = np.array([[1.0, 0.0], [0.0, 1.0], [1.0, 0.0], [2.0, 0.0]])
    q = np.array([[1.0, 0.0], [1.5, 0.0], [0.0, 0.0]])
    idx, d2 = orc.l2_argmin(q, g)
    np.testing.assert_array_equal(idx, [0, 0, 0])
    np.testing.assert_allclose(d2, [0.0, 0.25, 1.0])


def test_cov_branch_fit_equals_svd_restatement():
    """pca_cov_fit (covariance + eigh, useless/train.py:97-103, used for the C3-shape
    fixture) == pca_full_fit (the SVD restatement pinned by the reference's own
    train-v4.py output) on an n >= d standardised problem."""
    x = orc.int_synth_faces(900, 16, r=40, seed=4)
    a = orc.pca_cov_fit(x, 20)
    mu, _, sc = orc.standard_scaler_fit(x)
    b = orc.pca_full_fit((x - mu) / sc, 20)
    np.testing.assert_allclose(a["explained_variance_"], b["explained_variance_"], rtol=1e-10)
    np.testing.assert_allclose(a["components_"], b["components_"], atol=1e-9)
    np.testing.assert_allclose(a["fit_transform"], b["fit_transform"], atol=1e-8)
    np.testing.assert_allclose(a["total_var"], b["total_var"], rtol=1e-12)


def test_int_synth_is_exact_and_sliceable():
    """The C3 fixture generator: integer-exact (same pixels for any BLAS), row slices
    regenerate identically, and the fixture's first rows have not drifted."""
    x = orc.int_synth_faces(5000, 128, r=160, seed=0, rows=(0, 64))
    y = orc.int_synth_faces(5000, 128, r=160, seed=0, rows=(32, 4100))
    np.testing.assert_array_equal(x[32:], y[:32])
    g = golden("fit_c3.npz")
    assert int(g["n"]) == 20000 and int(g["side"]) == 128
    # the fixture's scaler mean pins all 20000 rows; spot-check the generator on 64 rows
    assert x.dtype == np.uint8 and 100 < x.mean() < 200 and x.std() > 10


def test_oracle_manual_pca_on_light_like_hard_spectrum():
    """The oracle's manual_pca restatement against the reference's own manual_pca output
    on the Light-like clustered-gap set (tests/golden/fit_hard.npz): eigenvalues and all
    50 sign-normalised components."""
    g = golden("fit_hard.npz")
    x = orc.int_synth_faces(int(g["n"]), int(g["side"]), r=int(g["r"]), seed=int(g["seed"]),
                            spectrum=g["spectrum"])
    eig, mean, proj, lam = orc.manual_pca(x, int(g["k"]))
    np.testing.assert_allclose(lam, g["eigenvalues"], rtol=1e-10)
    np.testing.assert_allclose(mean.sum(), float(g["mean_sum"]), rtol=1e-14)
    comps = eig.T
    comps = comps * np.sign(comps[np.arange(len(comps)), np.argmax(np.abs(comps), axis=1)])[:, None]
    R = np.random.default_rng([5]).integers(0, 2, size=(x.shape[1], 8)).astype(np.float64) * 2.0 - 1.0
    np.testing.assert_allclose(comps @ R, g["comps_R"], atol=1e-8)
    np.testing.assert_allclose(comps[:, g["px"]], g["comps_px"], atol=1e-10)


def test_oracle_exact_light_spectrum():
    """The oracle's manual_pca on the committed real Light eigenvalues (the GPU test
    test_gpu_manual.py::test_fit_exact_light_spectrum's construction, smaller d)."""
    st = golden("light_stats.npz")
    lam_ref = st["eigenvalues"]
    n, k = int(st["n"]), len(lam_ref)
    r = n - 1
    lam = np.concatenate([lam_ref, lam_ref[-1] * np.geomspace(0.97, 1e-3, r - k)])
    rng = np.random.default_rng(2029)
    U = np.linalg.qr(rng.standard_normal((n, r)))[0]
    U = np.linalg.qr(U - U.mean(0))[0]
    V = np.linalg.qr(rng.standard_normal((1024, r)))[0]
    X = (U * np.sqrt((n - 1) * lam)) @ V.T + 100.0
    _, _, _, got = orc.manual_pca(X, k)
    np.testing.assert_allclose(got, lam_ref, rtol=1e-10)
    np.testing.assert_allclose(orc.manual_model_info_evr(got), st["evr_json"], atol=1e-10)
