"""Projection kernel (p - mean).W against the fp64 oracle."""
import numpy as np
import pytest

from oracle import eigenface_oracle as orc

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("d,k", [(4096, 16), (10000, 50), (16384, 128), (1000, 96), (333, 10),
                                 (4096, 200), (8192, 512)])
@pytest.mark.parametrize("b", [1, 300])
def test_project_u8(eng, d, k, b):
    rng = np.random.default_rng(d + k + b)
    mu = rng.uniform(60, 200, d).astype(np.float32)
    w = (rng.standard_normal((d, k)) / np.sqrt(d)).astype(np.float32)
    p = rng.integers(0, 256, (b, d), dtype=np.uint8)
    eng.set_model(mu, w)
    f = eng.project(p)
    ref = orc.project(p, mu.astype(np.float64), w.astype(np.float64))
    bound = np.abs(p.astype(np.float64) - mu) @ np.abs(w.astype(np.float64))
    assert f.shape == (b, k)
    assert np.all(np.abs(f - ref) <= 2e-6 * bound + 1e-6)


def test_project_f32(eng):
    rng = np.random.default_rng(3)
    d, k, b = 4096, 64, 129
    mu = rng.uniform(0, 1, d).astype(np.float32)
    w = rng.standard_normal((d, k)).astype(np.float32)
    p = rng.uniform(0, 1, (b, d)).astype(np.float32)
    eng.set_model(mu, w)
    f = eng.project(p)
    ref = orc.project(p, mu, w)
    bound = np.abs(p.astype(np.float64) - mu) @ np.abs(w.astype(np.float64))
    assert np.all(np.abs(f - ref) <= 2e-6 * bound + 1e-6)


def test_recognize_fused_matches_project_then_search(eng):
    rng = np.random.default_rng(4)
    d, k = 4096, 64
    mu = rng.uniform(60, 200, d).astype(np.float32)
    w = (rng.standard_normal((d, k)) / 64).astype(np.float32)
    gal = rng.integers(0, 256, (2000, d), dtype=np.uint8)
    eng.set_model(mu, w)
    g = eng.project(gal)
    eng.set_gallery(g)
    probes = np.clip(gal[:300].astype(np.int32) + rng.integers(-3, 4, (300, d)), 0, 255).astype(np.uint8)
    idx, best, feats = eng.recognize(probes, "l2", return_features=True)
    np.testing.assert_array_equal(idx, np.arange(300))
    f2 = eng.project(probes)
    np.testing.assert_array_equal(feats, f2)
    idx2, best2 = eng.search(f2, "l2")
    np.testing.assert_array_equal(idx, idx2)
    np.testing.assert_array_equal(best, best2)


def test_recognize_fused_wide_k(eng):
    """k = 512 (config 5 width): fused projection + wide search == planted identities."""
    rng = np.random.default_rng(14)
    d, k = 4096, 512
    mu = rng.uniform(60, 200, d).astype(np.float32)
    w = np.linalg.qr(rng.standard_normal((d, k)))[0].astype(np.float32)
    gal = rng.integers(0, 256, (3000, d), dtype=np.uint8)
    eng.set_model(mu, w)
    eng.set_gallery(eng.project(gal))
    probes = np.clip(gal[::10].astype(np.int32) + rng.integers(-3, 4, (300, d)), 0, 255).astype(np.uint8)
    for metric in ("l2", "cosine"):
        idx, _ = eng.recognize(probes, metric)
        np.testing.assert_array_equal(idx, np.arange(0, 3000, 10))


BF16_REL = 2.0 ** -8  # stated tolerance: |f_bf16 - f| <= 2^-8 * sum_px |p - round(mean)| |W| (+ fp32 term)


@pytest.mark.parametrize("d,k,b,mean_lo,mean_hi", [
    (4096, 64, 300, 60, 200),      # frag kernel, 128-column tiles (512 probes per workgroup)
    (10000, 200, 129, 60, 200),    # d % 64 != 0: the 128 x 128 kernel
    (65536, 512, 256, 60, 200),    # config 5: frag kernel, 512-column tiles, 128-pixel stages
    (8192, 256, 257, 60, 200),     # ragged batch through the frag kernel (256 x 256 tiles)
    (4160, 512, 300, 60, 200),     # d % 128 != 0 at 512 columns: 64-pixel stages, ragged batch
    (8192, 1024, 130, 60, 200),    # two 512-column tiles
    (4096, 128, 200, -40, 300)])   # round(mean) outside 0..255: the byte-mean wide kernel is skipped
def test_project_bf16_tolerance(eng, d, k, b, mean_lo, mean_hi):
    """Config 5 bf16 projection: uint8 pixels minus round(mean) are exact in bf16, so the
    error is W's bf16 rounding only (unit roundoff 2^-9), bounded per feature."""
    rng = np.random.default_rng(d + k)
    mu = rng.uniform(mean_lo, mean_hi, d).astype(np.float32)
    w = (rng.standard_normal((d, k)) / np.sqrt(d)).astype(np.float32)
    p = rng.integers(0, 256, (b, d), dtype=np.uint8)
    eng.set_model(mu, w, precision="bf16")
    f = eng.project(p)
    ref = orc.project(p, mu.astype(np.float64), w.astype(np.float64))
    a = np.abs(p.astype(np.float64) - np.rint(mu))
    # |p - round(mean)| > 256 (a mean outside 0..255) is itself rounded to bf16: twice the bound
    rounds = 1.0 if a.max() <= 256 else 2.0
    bound = rounds * BF16_REL * (a @ np.abs(w.astype(np.float64))) \
        + 2e-6 * (np.abs(p.astype(np.float64) - mu) @ np.abs(w.astype(np.float64))) + 1e-5
    err = np.abs(f - ref)
    assert np.all(err <= bound)
    # typical error is far below the bound (random-walk of the W roundings)
    rel = np.linalg.norm(f - ref) / np.linalg.norm(ref)
    assert rel < 4e-3, rel


def test_recognize_bf16_agrees_with_fp32(eng):
    """bf16 projection + fp32 search: argmin identity agreement with the fp32 path
    (planted probes, config-5 width k=512)."""
    rng = np.random.default_rng(21)
    d, k, n = 16384, 512, 4000
    mu = rng.uniform(60, 200, d).astype(np.float32)
    w = np.linalg.qr(rng.standard_normal((d, k)))[0].astype(np.float32)
    gal = rng.integers(0, 256, (n, d), dtype=np.uint8)
    eng.set_model(mu, w)
    eng.set_gallery(eng.project(gal))
    probes = np.clip(gal[:512].astype(np.int32) + rng.integers(-8, 9, (512, d)), 0, 255).astype(np.uint8)
    idx32, _ = eng.recognize(probes, "l2")
    eng.set_model(mu, w, precision="bf16")
    idx16, _ = eng.recognize(probes, "l2")
    np.testing.assert_array_equal(idx32, np.arange(512))
    np.testing.assert_array_equal(idx16, idx32)
