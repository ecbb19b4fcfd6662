"""Projection kernel (p - mean).W against the fp64 oracle."""
import numpy as np
import pytest

from oracle import eigenface_oracle as orc

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("d,k", [(4096, 16), (10000, 50), (16384, 128), (1000, 96), (333, 10)])
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
