"""GPU fit (mean, covariance, eigensolve, back-projection) against the reference
goldens and the oracle."""
import numpy as np
import pytest

from conftest import golden, local_golden
from oracle import eigenface_oracle as orc

pytestmark = pytest.mark.gpu


def _align(a, ref, axis=0):
    s = np.sign((a * ref).sum(axis=axis, keepdims=True))
    s[s == 0] = 1
    return a * s


def test_manual_pca_light_golden():
    """Real faces (faces/Light_version, 229 x 10000) through the GPU manual_pca vs the
    reference's own manual_pca output (useless/train.py:56-128)."""
    from eigenface import manual_pca
    g = local_golden("light_manual_pca.npz")
    eig, mean, proj, lam = manual_pca(g["X"], 50)
    assert eig.shape == (10000, 50) and proj.shape == (229, 50) and lam.shape == (50,)
    np.testing.assert_allclose(mean, g["mean_face"], rtol=1e-15)
    np.testing.assert_allclose(lam, g["eigenvalues"], rtol=1e-9)
    e10 = _align(eig[:, :10], g["eigenfaces_10"].astype(np.float64))
    np.testing.assert_allclose(e10, g["eigenfaces_10"], atol=1e-6)
    p = _align(proj, g["projected"])
    np.testing.assert_allclose(p, g["projected"], rtol=1e-6, atol=1e-6 * np.abs(g["projected"]).max())
    np.testing.assert_allclose(orc.manual_model_info_evr(lam), g["evr_json"], atol=1e-10)
    # all 50 eigenfaces against the oracle, 1e-4 relative (north-star tolerance)
    o_eig, _, _, _ = orc.manual_pca(g["X"], 50)
    np.testing.assert_allclose(_align(eig, o_eig), o_eig, atol=1e-4 * np.abs(o_eig).max())


def test_sklearn_path_golden():
    """train-v4.py's StandardScaler + PCA (solver pinned 'full') vs the GPU fit."""
    from eigenface import EigenfacePCA
    g = golden("sklearn_path.npz")
    m = EigenfacePCA(16, standardize=True).fit(g["X"])
    np.testing.assert_allclose(m.scaler_mean_, g["scaler_mean"], rtol=1e-14)
    np.testing.assert_allclose(m.scaler_var_, g["scaler_var"], rtol=1e-10)
    np.testing.assert_allclose(m.scaler_scale_, g["scaler_scale"], rtol=1e-10)
    np.testing.assert_allclose(m.explained_variance_, g["explained_variance"], rtol=1e-9)
    np.testing.assert_allclose(m.explained_variance_ratio_, g["explained_variance_ratio"], rtol=1e-9)
    np.testing.assert_allclose(m.singular_values_, g["singular_values"], rtol=1e-9)
    np.testing.assert_allclose(m.noise_variance_, g["noise_variance"], rtol=1e-8)
    # deterministic sign rule == sklearn svd_flip: no alignment needed
    np.testing.assert_allclose(m.components_, g["components"], atol=1e-8)
    np.testing.assert_allclose(m.face_features_, g["face_features"], rtol=1e-6,
                               atol=1e-7 * np.abs(g["face_features"]).max())
    np.testing.assert_allclose(m.mean_face_, g["mean_face"], rtol=1e-14)
    f = m.transform(g["probes"])
    np.testing.assert_allclose(f, g["probe_features"], rtol=1e-5, atol=1e-4)
    idx, sim = m.recognize(g["probes"], "cosine", threshold=float(g["threshold"]))
    pid = np.where(idx >= 0, g["labels"][np.maximum(idx, 0)], -1)
    np.testing.assert_array_equal(pid, g["probe_person_id"])
    np.testing.assert_allclose(sim, g["probe_similarity"], atol=1e-5)


@pytest.mark.parametrize("n,d,k,r", [
    (60, 4096, 20, 32), (87, 1000, 86, 32), (500, 64, 10, 32), (300, 48, 48, 32),
    # k > 80: direct grid-Jacobi (order <= 1024) and subspace iteration + grid Jacobi
    (600, 4096, 128, 256), (1500, 4096, 100, 256), (3000, 1024, 130, 256),
    # order >= 2048: the 256 x 384 SYRK tiles, ragged against both tile sizes (Gram, covariance)
    (2100, 4096, 20, 32), (2500, 2116, 20, 32),
    # covariance path with n > 65536: the int8 product's int32 -> int64 flush
    (70000, 256, 12, 64),
    # covariance path with d % 4 != 0: byte-granular transpose + separate column stats
    (400, 50, 10, 32), (131009, 36, 6, 16)])
def test_fit_shapes_vs_oracle(n, d, k, r):
    """Direct-Jacobi (order <= 88), Gram and covariance (n >= d) branches, exact int8
    covariance, wide k."""
    from eigenface import manual_pca
    side = int(np.sqrt(d))
    if side * side == d:
        x, _ = orc.synth_faces(n, side, r=min(r, d), seed=n + d)
    else:
        x = np.random.default_rng(n).integers(0, 256, (n, d), dtype=np.uint8)
    eig, mean, proj, lam = manual_pca(x, k)
    o_eig, o_mean, o_proj, o_lam = orc.manual_pca(x, k)
    kk = o_lam.shape[0]
    assert lam.shape == (kk,)
    np.testing.assert_allclose(mean, o_mean, rtol=1e-14)
    keep = o_lam > 1e-9 * o_lam[0]
    np.testing.assert_allclose(lam[keep], o_lam[keep], rtol=1e-8)
    # compare eigenvectors with a clear gap only
    gap = np.ones(kk, bool)
    rel = np.abs(np.diff(o_lam)) / o_lam[0]
    gap[:-1] &= rel > 1e-6
    gap[1:] &= rel > 1e-6
    gap &= keep
    a = _align(eig, o_eig)
    np.testing.assert_allclose(a[:, gap], o_eig[:, gap], atol=1e-6)


@pytest.mark.parametrize("n,d", [(5000, 4096), (4096, 6400)])
def test_fit_int8_digit_products(n, d):
    """The fine-phase products C.Q as exact int8 digit pairs (launch_cq_i8, ef_proj_i8.hip:
    block width 256 = 2k, order a multiple of 2048) on an unstandardised covariance
    (n >= d) and Gram (n < d) whose rows span very different scales: 64 constant pixels
    (zero rows: scale exponent 0, all digits 0) and 64 pixels of 1/16 the contrast (the
    per-row scaling keeps their digits full) — against the oracle's fp64 eigh
    (useless/train.py:82-116)."""
    from eigenface import manual_pca
    side = int(np.sqrt(d))
    x, _ = orc.synth_faces(n, side, r=64, seed=n + 7)
    x[:, :64] = 3
    x[:, 64:128] //= 16
    eig, mean, proj, lam = manual_pca(x, 128)
    o_eig, o_mean, o_proj, o_lam = orc.manual_pca(x, 128)
    keep = o_lam > 1e-9 * o_lam[0]
    np.testing.assert_allclose(lam[keep], o_lam[keep], rtol=1e-8)
    gap = np.ones(o_lam.shape[0], bool)
    rel = np.abs(np.diff(o_lam)) / o_lam[0]
    gap[:-1] &= rel > 1e-6
    gap[1:] &= rel > 1e-6
    gap &= keep
    assert gap.sum() >= 32
    a = _align(eig, o_eig)
    np.testing.assert_allclose(a[:, gap], o_eig[:, gap], atol=1e-6)


def test_subspace_rank_deficient_block_retries_checked():
    """A block wider than the data's rank (order 2116, k = 50 -> block 100, rank 40): the
    CholQR factor fails in the first iterations.  The fit defers that check to its
    Rayleigh-Ritz steps, finds the failure there, and reruns with the per-iteration check,
    whose rank-deficient fallback (eigen-orthonormalisation) completes it: the spectrum
    equals the oracle's (40 non-zero eigenvalues, the rest at the rounding floor)."""
    from eigenface import manual_pca
    base, _ = orc.synth_faces(40, 46, r=32, seed=9)
    x = np.concatenate([base] * 75)  # 3000 x 2116, rank <= 40
    eig, mean, proj, lam = manual_pca(x, 50)
    o_eig, o_mean, o_proj, o_lam = orc.manual_pca(x, 50)
    assert np.all(np.isfinite(eig)) and np.all(np.isfinite(lam))
    keep = o_lam > 1e-9 * o_lam[0]
    assert keep.sum() <= 40
    np.testing.assert_allclose(lam[keep], o_lam[keep], rtol=1e-8)
    assert np.all(np.abs(lam[~keep]) <= 1e-7 * o_lam[0])


def test_rank_deficient_duplicates():
    """Duplicate faces make the Gram singular; the fit must stay finite and
    reproduce the non-zero spectrum."""
    from eigenface import manual_pca
    x, _ = orc.synth_faces(40, 32, r=8, seed=2)
    x = np.concatenate([x, x, x])  # 120 x 1024, rank <= 40
    eig, mean, proj, lam = manual_pca(x, 20)
    o_eig, _, _, o_lam = orc.manual_pca(x, 20)
    assert np.all(np.isfinite(eig)) and np.all(np.isfinite(proj))
    np.testing.assert_allclose(lam, o_lam, rtol=1e-8)


def test_standardized_covariance_path_vs_oracle():
    """StandardScaler + PCA with n >= d: the int8 covariance scaled by 1/scale_i 1/scale_j
    (train-v4.py:131-134) vs the oracle's sklearn 'full' restatement."""
    from eigenface import EigenfacePCA
    x, _ = orc.synth_faces(3000, 16, r=64, seed=11)
    x[:, 0] = 7  # a constant pixel: StandardScaler scale 1
    m = EigenfacePCA(12, standardize=True).fit(x)
    o = orc.train_pca_model(x, 12)
    np.testing.assert_allclose(m.explained_variance_, o["pca"]["explained_variance_"], rtol=1e-9)
    np.testing.assert_allclose(m.components_, o["pca"]["components_"], atol=1e-8)
    np.testing.assert_allclose(m.face_features_, o["face_features"], rtol=1e-6,
                               atol=1e-7 * np.abs(o["face_features"]).max())


@pytest.mark.parametrize("side", [8, 46])
def test_covariance_multi_pass(side):
    """Force the int8 covariance into several syrk passes (slab budget of one split,
    EF_OPT_COV_SLAB_BYTES): the int64 slab accumulation between passes must keep the
    product exact (order 64: 256 x 256 tiles; order 2116: 256 x 384 tiles)."""
    from eigenface import get_engine, manual_pca
    x, _ = orc.synth_faces(140_000, side, r=32, seed=5)  # K = 140000 > 2047 * 64 samples per split
    e = get_engine(0)
    default = e.get_option("cov_slab_bytes")
    e.set_option("cov_slab_bytes", side ** 4 * 4)
    try:
        eig, mean, proj, lam = manual_pca(x, 8)
    finally:
        e.set_option("cov_slab_bytes", default)
    o_eig, o_mean, _, o_lam = orc.manual_pca(x, 8)
    np.testing.assert_allclose(mean, o_mean, rtol=1e-14)
    np.testing.assert_allclose(lam, o_lam, rtol=1e-9)
    np.testing.assert_allclose(_align(eig, o_eig), o_eig, atol=1e-6)


@pytest.mark.parametrize("n,side,k,std", [(3000, 16, 12, False), (700, 32, 40, True), (5000, 8, 64, True)])
def test_training_projection_int8_digits(n, side, k, std):
    """F = ((X - mu) w) E through the int8 digit GEMM (ef_proj_i8.hip) equals the fp64
    CPU restatement of the centred, scaled product to fp64 rounding (useless/train.py:122,
    train-v4.py:134)."""
    from eigenface import EigenfacePCA
    x, _ = orc.synth_faces(n, side, r=min(48, side * side), seed=n + side)
    m = EigenfacePCA(k, standardize=std).fit(x)
    f8 = m.face_features_
    z = (x - m.scaler_mean_) / m.scaler_scale_ if std else x - m.mean_face_
    ref = z @ m.components_.T
    np.testing.assert_allclose(f8, ref, rtol=0, atol=1e-11 * np.abs(ref).max())


def test_pooled_workspaces_refit_and_trim():
    """ef_fit reuses the context's pooled workspaces across calls of different shapes
    (grow-only slots) and ef_trim frees them; results stay identical to a fresh context."""
    from eigenface import Engine
    xa, _ = orc.synth_faces(900, 16, r=32, seed=21)   # covariance path
    xb, _ = orc.synth_faces(120, 32, r=32, seed=22)   # Gram path
    with Engine(0) as e:
        ra1 = e.fit(xa, 10)
        rb1 = e.fit(xb, 10)
        ra2 = e.fit(xa, 10)
        e.trim()
        rb2 = e.fit(xb, 10)
    with Engine(0) as f:
        ra3 = f.fit(xa, 10)
    np.testing.assert_array_equal(ra1.components, ra2.components)
    np.testing.assert_array_equal(ra1.components, ra3.components)
    np.testing.assert_array_equal(rb1.components, rb2.components)
    np.testing.assert_array_equal(ra1.projection, ra3.projection)


def test_syrk_timing_hook():
    """EF_KERNEL_SYRK: one hipEvent pair per fit around the int8 SYRK launches (the fit
    roofline's duration in bench.py); nothing recorded while timing is off."""
    from eigenface import Engine
    x, _ = orc.synth_faces(900, 16, r=32, seed=23)
    with Engine(0) as e:
        e.fit(x, 10)
        assert e.timing_get("syrk") == (0.0, 0)
        e.timing(True)
        r1 = e.fit(x, 10)
        e.fit(x, 10)
        ms, n = e.timing_get("syrk")
        assert n == 2 and ms > 0
        e.timing_reset()
        assert e.timing_get("syrk") == (0.0, 0)
        r2 = e.fit(x, 10)
    np.testing.assert_array_equal(r1.components, r2.components)


def test_eigensolver_non_convergence_is_reported():
    """The subspace iteration's cap (EF_OPT_FIT_MAX_ITERS) ends an unconverged solve with
    EF_E_NUMERIC instead of returning partial eigenpairs; FaceTrainer.train_pca_model
    maps it to False with a message, as train-v4.py:114-120 does for a failed fit."""
    from eigenface import EigenfaceError, get_engine
    from eigenface._native import EF_E_NUMERIC
    from eigenface.compat import FaceTrainer
    x, _ = orc.synth_faces(600, 64, r=256, seed=31)  # Gram path, order 600 > 88: subspace iteration
    e = get_engine(0)
    e.set_option("fit_max_iters", 2)
    try:
        with pytest.raises(EigenfaceError) as ei:
            e.fit(x, 40)
        assert ei.value.code == EF_E_NUMERIC and "did not converge" in str(ei.value)
        tr = FaceTrainer(n_components=40)
        tr.face_images = x
        tr.face_labels = np.zeros(len(x), np.int64)
        assert tr.train_pca_model() is False and not tr.is_trained
    finally:
        e.set_option("fit_max_iters", 500)
    r = e.fit(x, 40)  # default cap: converges
    assert r.iters > 2


def _c3_fixture():
    g = golden("fit_c3.npz")
    x = orc.int_synth_faces(int(g["n"]), int(g["side"]), r=int(g["r"]), seed=int(g["seed"]))
    return g, x


@pytest.mark.parametrize("cheb", [1, 0])
@pytest.mark.parametrize("coarse_fp32", [1, 2, 0])
def test_fit_c3_shape_vs_oracle(coarse_fp32, cheb):
    """The C3 fit shape (d = 128 x 128 = 16384, k = 128, n = 20000 >= d, StandardScaler):
    covariance branch at order 16384, the Rayleigh-Ritz schedule, the coarse phase
    (coarse_fp32 = 1, the default: split-bf16 matrix-core products; 2: fp32 products; 0:
    fp64 throughout) and the Chebyshev recurrence (cheb = 1, the default) or plain shifted
    steps, against the oracle's covariance-branch fit (tests/golden/make_fit_c3.py;
    exact-integer generator, so the box regenerates the same pixels).  Eigenvalues rtol
    1e-9, components 1e-4 relative (north star)."""
    from eigenface import get_engine
    g, x = _c3_fixture()
    e = get_engine(0)
    e.set_option("fit_fp32_coarse", coarse_fp32)
    e.set_option("fit_chebyshev", cheb)
    try:
        r = e.fit(x, int(g["k"]), standardize=True)
    finally:
        e.set_option("fit_fp32_coarse", 1)
        e.set_option("fit_chebyshev", 1)
    assert r.k == 128 and r.iters > 0  # subspace iteration, not the direct Jacobi
    np.testing.assert_allclose(r.mean, g["scaler_mean"], rtol=1e-14)
    np.testing.assert_allclose(r.scale, g["scaler_scale"], rtol=1e-12)
    np.testing.assert_allclose(r.total_var, float(g["total_var"]), rtol=1e-12)
    np.testing.assert_allclose(r.eigenvalues, g["eigenvalues"], rtol=1e-9)
    R, px = _c3_probe_matrices(x.shape[1])
    np.testing.assert_array_equal(px, g["px"])
    cr = r.components @ R
    s = np.sign((cr * g["comps_R"]).sum(axis=1))  # sign-align, then account for every flip
    # sklearn's svd_flip (extmath.py:946-952) makes each component's largest-|.| entry
    # positive.  A component may come out with the other sign only when its two largest
    # |entries| (oracle: pixels i1, i2, values v1 > 0, v2) are tied within the two
    # fits' difference at those pixels: then the GPU's own largest entry is i2 and it
    # chose the sign from there.  Anything else is a sign-rule bug.
    ti, tv = g["top_idx"], g["top_val"]
    flips = []
    for c in np.nonzero(s < 0)[0]:
        gv = -r.components[c, ti[c]]  # GPU values at i1, i2 after alignment
        err = np.abs(gv - tv[c]).sum()
        margin = abs(tv[c, 0]) - abs(tv[c, 1])
        flips.append((int(c), float(margin), float(err)))
        assert margin <= err + 1e-15, f"component {c}: sign flipped with a clear max entry (margin {margin:.3e})"
        assert int(np.argmax(np.abs(r.components[c]))) == int(ti[c, 1]), f"component {c}"
        assert r.components[c, ti[c, 1]] > 0
    print(f"C3 fit (coarse={coarse_fp32}, chebyshev={cheb}, {r.iters} iterations): {len(flips)} svd_flip sign(s) differ from the oracle's, "
          f"all at near-tied max entries (component, margin, fit difference): {flips}")
    cr *= s[:, None]
    # unit rows against +-1 columns: |c.R| ~ 1, so atol 1e-4 is the 1e-4 relative bar
    np.testing.assert_allclose(cr, g["comps_R"], atol=1e-4)
    np.testing.assert_allclose(r.components[:, px] * s[:, None], g["comps_px"], atol=1e-4 * np.abs(g["comps_px"]).max())
    f = r.projection[:64] * s[None, :]
    np.testing.assert_allclose(f, g["features"], rtol=0, atol=1e-4 * np.abs(g["features"]).max())


def _c3_probe_matrices(d):
    r = np.random.default_rng([5]).integers(0, 2, size=(d, 8)).astype(np.float64) * 2.0 - 1.0
    px = np.sort(np.random.default_rng([6]).choice(d, size=256, replace=False))
    return r, px


def test_fused_column_stats_exact_beyond_32bit_quarters():
    """transpose_stats_lds_kernel (d % 256 == 0, covariance path): a workgroup covers
    nkb / 128 blocks of 64 samples; past ~1060 blocks the four sample quarters' Σx² of one
    pixel exceed 2^32 together (near-255 pixels), so they are added in 64 bits.  n = 9M
    samples (1100 blocks per workgroup) vs exact integer sums: StandardScaler mean and var
    (train-v4.py:131) to the last bits."""
    import torch
    from eigenface import get_engine
    n, d = 9_000_000, 256
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.randint(249, 256, (n, d), dtype=torch.uint8, device="cuda", generator=g)
    s1 = torch.zeros(d, dtype=torch.int64, device="cuda")
    s2 = torch.zeros(d, dtype=torch.int64, device="cuda")
    for i in range(0, n, 1 << 20):
        c = x[i:i + (1 << 20)].to(torch.int64)
        s1 += c.sum(0)
        s2 += (c * c).sum(0)
    s1, s2 = [int(v) for v in s1.cpu()], [int(v) for v in s2.cpu()]
    assert max(s2) // 128 > (1 << 32)  # one workgroup's share of Σx² needs 64 bits
    r = get_engine(0).fit(x, 100, standardize=True, projection=False)  # k > 80: direct Jacobi
    mean, var = r.mean.cpu().numpy(), r.var.cpu().numpy()
    from fractions import Fraction
    m_ref = np.array([float(Fraction(a, n)) for a in s1])
    v_ref = np.array([float(Fraction(n * b - a * a, n * n)) for a, b in zip(s1, s2)])
    np.testing.assert_allclose(mean, m_ref, rtol=1e-15)
    np.testing.assert_allclose(var, v_ref, rtol=1e-12)
    del x
    torch.cuda.empty_cache()


def _signs_vs_fixture(comps, g):
    """Per-component sign alignment against a fixture's sign-normalised components (the
    svd_flip rule: largest |entry| positive), accounting for every flip: allowed only
    where the fixture's two largest |entries| are tied within the fits' difference there
    (then the GPU's own largest entry is the runner-up pixel).  Returns the signs."""
    R, px = _c3_probe_matrices(comps.shape[1])
    np.testing.assert_array_equal(px, g["px"])
    s = np.sign(((comps @ R) * g["comps_R"]).sum(axis=1))
    ti, tv = g["top_idx"], g["top_val"]
    for c in np.nonzero(s < 0)[0]:
        gv = -comps[c, ti[c]]
        margin = abs(tv[c, 0]) - abs(tv[c, 1])
        assert margin <= np.abs(gv - tv[c]).sum() + 1e-15, f"component {c}: sign flipped with a clear max entry"
        assert int(np.argmax(np.abs(comps[c]))) == int(ti[c, 1]) and comps[c, ti[c, 1]] > 0
    return s


@pytest.mark.parametrize("name", ["fit_hard", "fit_c2"])
def test_fit_vs_reference_manual_pca(name):
    """manual_pca (useless/train.py:56-128) on the GPU vs the REFERENCE's own manual_pca
    run on the same exact-integer synthetic pixels (tests/golden/make_goldens.py
    fit_shapes; the box regenerates them bit for bit):

    * fit_hard: n = 229, d = 100 x 100 (faces/Light_version's shape) with the real Light
      set's eigenvalue profile, so its sample spectrum has the real set's clustered gaps
      (min relative gap 1.1 %): ALL 50 components at the north star's 1e-4 relative;
    * fit_c2: BASELINE.json configs[1]'s fit shape, n = 10000, d = 16384, k = 64: the Gram
      path at order 10000 (int8 Gram, subspace iteration, A^T.V back-projection).

    Eigenvalues rtol 1e-9; unit components through a +-1 probe matrix (|c.R| ~ |c| = 1, so
    atol 1e-4 is 1e-4 relative) and at 256 pixels; projections 1e-4 of their scale."""
    from eigenface import manual_pca
    g = golden(name + ".npz")
    spec = g["spectrum"] if "spectrum" in g.files else None
    x = orc.int_synth_faces(int(g["n"]), int(g["side"]), r=int(g["r"]), seed=int(g["seed"]), spectrum=spec)
    k = int(g["k"])
    eig, mean, proj, lam = manual_pca(x, k)
    assert eig.shape == (x.shape[1], k) and proj.shape == (x.shape[0], k)
    np.testing.assert_allclose(mean.sum(), float(g["mean_sum"]), rtol=1e-13)
    np.testing.assert_allclose(lam, g["eigenvalues"], rtol=1e-9)
    comps = eig.T
    s = _signs_vs_fixture(comps, g)
    R, px = _c3_probe_matrices(x.shape[1])
    err_r = np.abs((comps @ R) * s[:, None] - g["comps_R"]).max()
    err_px = np.abs(comps[:, px] * s[:, None] - g["comps_px"]).max()
    f = proj[:64] * s[None, :]
    err_f = np.abs(f - g["projected"]).max() / np.abs(g["projected"]).max()
    print(f"{name}: {k} components, max |dc.R| {err_r:.2e}, max |dc| at 256 px {err_px:.2e}, "
          f"projection rel {err_f:.2e}, flips {int((s < 0).sum())}")
    assert err_r <= 1e-4 and err_px <= 1e-4 and err_f <= 1e-4
    np.testing.assert_allclose(np.linalg.norm(proj, axis=0), g["proj_colnorm"], rtol=1e-8)


def test_fit_c3_full_size_properties():
    """The 1M-face C3 fit itself (train-v4.py:126-146 at n = 1M, d = 16384, k = 128: the
    8 K-split int32 SYRK slabs at <= 131,008 samples each, the order-16384 subspace
    iteration), checked by properties no fixture can hold at this size, with an
    independent fp64 checker (torch fp64 GEMMs on the GPU over the standardised data
    Z = (X - mean) / scale, streamed in chunks):

    * components orthonormal (|V^T V - I| <= 1e-10);
    * Rayleigh quotients v^T C v equal the returned eigenvalues (rtol 1e-9);
    * residuals |C v - lambda v| <= 1e-9 lambda_1 for every component (the engine's own
      criterion, ef_fit.hip fit_resid_tol; round 5 asserted only 1e-6);
    * per component |r_i| / gap_i <= 1e-4, gap_i to the nearest other eigenvalue: the
      eigenvector error bound (Davis-Kahan).  The fit is run at k = 136 as well, so the gap
      of component 128 to lambda_129 is known; both fits are checked;
    * mean / scale equal exact integer column statistics."""
    import torch
    from eigenface import get_engine, synth
    n, side, k, r = 1_000_000, 128, 128, 256
    d = side * side
    dev = torch.device("cuda", 0)
    B = torch.from_numpy(synth.basis(d, r, 5)).to(dev, torch.float32)
    sp = torch.from_numpy(synth.spectrum(r)).to(dev, torch.float32)
    mu = torch.from_numpy(synth.mean_face(side)).to(dev, torch.float32)
    X = torch.empty((n, d), dtype=torch.uint8, device=dev)
    gen = torch.Generator(device=dev).manual_seed(77)
    for a in range(0, n, 32768):
        e = min(n, a + 32768)
        z = torch.randn((e - a, r), generator=gen, device=dev) * sp
        X[a:e] = (mu + z @ B.T + 2.0 * torch.randn((e - a, d), generator=gen, device=dev)).round_().clamp_(0, 255) \
            .to(torch.uint8)
    del B, z
    eng = get_engine(0)
    res_w = eng.fit(X, k + 8, standardize=True, projection=False)  # lambda_129.. for the gaps at 128
    res = eng.fit(X, k, standardize=True, projection=False)
    # exact column statistics
    s1 = torch.zeros(d, dtype=torch.float64, device=dev)
    s2 = torch.zeros(d, dtype=torch.float64, device=dev)
    for a in range(0, n, 65536):
        c = X[a:a + 65536].to(torch.float64)
        s1 += c.sum(0)
        s2 += (c * c).sum(0)
    m_ref = s1 / n
    var_ref = s2 / n - m_ref * m_ref
    torch.testing.assert_close(res.mean, m_ref, rtol=1e-13, atol=0)
    sc_ref = torch.where(var_ref > 0, var_ref.sqrt(), torch.ones_like(var_ref))
    torch.testing.assert_close(res.scale, sc_ref, rtol=1e-9, atol=0)
    inv = 1.0 / res.scale
    lam_all = res_w.eigenvalues  # k + 8 values: the spectrum the gaps are measured on
    torch.testing.assert_close(res.eigenvalues, lam_all[:k], rtol=1e-9, atol=0)
    for r_ in (res, res_w):
        V = r_.components.T.contiguous()  # d x kk fp64
        lam = r_.eigenvalues
        kk = V.shape[1]
        # C V = Z^T (Z V) / (n - 1), streamed
        CV = torch.zeros((d, kk), dtype=torch.float64, device=dev)
        for a in range(0, n, 32768):
            zc = (X[a:a + 32768].to(torch.float64) - res.mean) * inv
            CV += zc.T @ (zc @ V)
        CV /= n - 1
        orth = (V.T @ V - torch.eye(kk, dtype=torch.float64, device=dev)).abs().max().item()
        rq = (V * CV).sum(0)
        rq_err = ((rq - lam).abs() / lam).max().item()
        resid = (CV - V * lam).norm(dim=0)
        res_rel = (resid / lam[0]).max().item()
        # gap of component i to its nearest neighbour in the k + 8 spectrum (the last kept
        # column of the k + 8 fit has no right neighbour and is excluded)
        ng = min(kk, k + 7)
        la = lam_all
        gap = torch.minimum(torch.cat([la[:1] * 0 + float("inf"), la[:-1] - la[1:]])[:ng],
                            (la[:-1] - la[1:])[:ng])
        r_gap = (resid[:ng] / gap).max().item()
        print(f"C3 1M fit k={kk}: {r_.iters} iterations, |V'V-I| {orth:.2e}, Rayleigh rel {rq_err:.2e}, "
              f"max |Cv - lv| / l1 {res_rel:.2e}, max |r_i| / gap_i {r_gap:.2e} "
              f"(min gap {(gap.min() / la[0]).item():.2e} l1)")
        assert orth <= 1e-10
        assert rq_err <= 1e-9
        assert res_rel <= 1e-9
        assert r_gap <= 1e-4
        del CV
    del X
    torch.cuda.empty_cache()


def test_device_tensors_outlive_a_closed_engine():
    """Tensors that a device call marked as used on the engine's stream (record_stream, so
    the caching allocator does not hand them to another stream too early) are freed after
    the engine is closed: the engine's own stream is a process-lifetime torch pool stream,
    so the allocator's free-time event record cannot hit a destroyed stream (round 5: with
    a library-created stream this crashed the process at the tensor's free)."""
    import subprocess
    import sys
    from conftest import PKG
    code = (f"import sys; sys.path.insert(0, {PKG!r})\n"
            "import torch\n"
            "from eigenface import Engine\n"
            "from oracle import eigenface_oracle as orc\n"
            "x, _ = orc.synth_faces(600, 32, r=24, seed=2)\n"
            "X = torch.from_numpy(x).cuda()\n"
            "e = Engine(0)\n"
            "r = e.fit(X, 8, projection=True)\n"
            "e.set_model(r.mean.float().cpu().numpy(), r.components.T.float().contiguous().cpu().numpy())\n"
            "f = e.project(X)\n"
            "e.close()\n"
            "del X, f, r\n"
            "y = torch.ones(1 << 20, device='cuda').sum()\n"
            "torch.cuda.synchronize(); print('ok', float(y))\n")
    res = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240,
                         cwd=__import__("conftest").ROOT)
    assert res.returncode == 0, (res.returncode, res.stderr[-2000:])
    assert res.stdout.strip().startswith("ok")


@pytest.mark.parametrize("m", [1, 15, 17, 100, 255, 256])
def test_chol_inv_blocked_vs_fp64(eng, m):
    """the blocked CholQR factor (ef_chol_blk.hip, the default for every
    fit at m <= 256) checked directly, for odd orders and orders that pad the diagonal to a
    multiple of 16: Li equals numpy's fp64 inv(cholesky(G)) to 1e-12 of its scale, is lower
    triangular, and Li G Li^T = I to 1e-12."""
    rng = np.random.default_rng(m)
    A = rng.standard_normal((m + 12, m)) * np.geomspace(1.0, 1e-2, m)  # condition ~1e4
    G = A.T @ A
    Li, info = eng.chol_inv(G)
    assert info == 0
    ref = np.linalg.inv(np.linalg.cholesky(G))
    np.testing.assert_allclose(Li, ref, rtol=0, atol=1e-12 * np.abs(ref).max())
    assert np.all(np.triu(Li, 1) == 0.0)
    np.testing.assert_allclose(Li @ G @ Li.T, np.eye(m), rtol=0, atol=1e-10)  # ~ eps x cond(G) = 1e-12


@pytest.mark.parametrize("m,j", [(17, 9), (64, 0), (256, 200)])
def test_chol_inv_failed_pivot_leaves_li(eng, m, j):
    """The failed-pivot contract tri_inv_blk_kernel and the subspace iteration rely on:
    the first pivot <= tol x max diag(G) gives info = -(column + 1), and Li is left exactly
    as the caller gave it."""
    rng = np.random.default_rng(m + j)
    A = rng.standard_normal((m + 12, m))
    G = A.T @ A
    # make column j's pivot G[j,j] - |L^-1 G[:j, j]|^2 negative, leaving columns < j valid
    piv = G[j, j] - (np.sum(np.linalg.solve(np.linalg.cholesky(G[:j, :j]), G[:j, j]) ** 2) if j else 0.0)
    G[j, j] -= piv + 1.0
    sentinel = np.full((m, m), 7.25)
    Li, info = eng.chol_inv(G, Li=sentinel)
    assert info == -(j + 1)
    np.testing.assert_array_equal(Li, sentinel)
