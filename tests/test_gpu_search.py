"""Distance GEMM + fused arg-best (search kernel) against the fp64 oracle."""
import numpy as np
import pytest

from conftest import golden
from oracle import eigenface_oracle as orc
from parity_util import assert_exact_argbest

pytestmark = pytest.mark.gpu


def _check_l2(q, g, idx, best):
    """Exact fp64 first-argmin outside the engine's 1e-12 tie window (parity_util), and
    the reported distance is the chosen row's difference-form distance."""
    assert_exact_argbest(q, g, idx, "l2")
    d_gpu = ((q.astype(np.float64) - g[idx].astype(np.float64)) ** 2).sum(1)
    np.testing.assert_allclose(best, d_gpu, rtol=1e-6, atol=1e-30)


def _check_cos(q, g, idx, best):
    assert_exact_argbest(q, g, idx, "cosine")
    s_gpu = orc.cosine_scores(q, g)[np.arange(len(q)), idx]
    np.testing.assert_allclose(best, s_gpu, atol=2e-6)


@pytest.mark.parametrize("k", [8, 16, 50, 64, 96, 128, 200, 256, 300, 512])
@pytest.mark.parametrize("n,b", [(1, 3), (33, 257), (3001, 300)])
def test_l2_random(eng, k, n, b):
    rng = np.random.default_rng(k * 1000 + n)
    g = rng.standard_normal((n, k)).astype(np.float32)
    q = rng.standard_normal((b, k)).astype(np.float32)
    eng.set_gallery(g)
    idx, best = eng.search(q, "l2")
    _check_l2(q, g, idx, best)


@pytest.mark.parametrize("k", [256, 512])
@pytest.mark.parametrize("b", [1024, 2048, 4096])
def test_wide_xcd_block_deal(eng, k, b):
    """Batches of >= 8 wide probe tiles use the blocked (chunk x probe-tile) XCD deal
    (search_plan pblk/cblk); every pair must still be swept once: exact vs fp64, L2 and
    cosine, ragged last gallery tile."""
    rng = np.random.default_rng(k + b)
    n = 5003
    g = rng.standard_normal((n, k)).astype(np.float32)
    q = rng.standard_normal((b, k)).astype(np.float32)
    eng.set_gallery(g)
    idx, best = eng.search(q, "l2")
    _check_l2(q, g, idx, best)
    idx_c, best_c = eng.search(q, "cosine")
    _check_cos(q, g, idx_c, best_c)


@pytest.mark.parametrize("k", [16, 64, 128, 256, 512])
def test_cosine_random(eng, k):
    rng = np.random.default_rng(k)
    g = rng.standard_normal((4000, k)).astype(np.float32)
    q = rng.standard_normal((513, k)).astype(np.float32)
    eng.set_gallery(g)
    idx, best = eng.search(q, "cosine")
    _check_cos(q, g, idx, best)


def test_cosine_ties_and_zero_norm_golden(eng):
    """Reference tie-break (first max) and zero-norm handling, from
    scan-template-v4.py's recognize_face_with_model run on tests/golden/ties.npz."""
    t = golden("ties.npz")
    eng.set_gallery(t["gallery"].astype(np.float32))
    idx, sim = eng.search(t["probes"].astype(np.float32), "cosine")
    np.testing.assert_array_equal(idx, t["idx"])
    np.testing.assert_allclose(sim, t["sim"], atol=1e-6)


@pytest.mark.parametrize("k", [32, 512])
def test_l2_duplicates_lowest_index(eng, k):
    rng = np.random.default_rng(5)
    g = rng.standard_normal((1000, k)).astype(np.float32)
    g[700] = g[5]
    g[999] = g[5]
    g[300] = g[64]
    q = np.stack([g[5], g[999], g[64], g[300]])
    eng.set_gallery(g)
    idx, d = eng.search(q, "l2")
    np.testing.assert_array_equal(idx, [5, 5, 64, 64])
    np.testing.assert_array_equal(d, [0, 0, 0, 0])


def test_empty_gallery(eng):
    eng.set_gallery(np.zeros((0, 16), np.float32))
    idx, best = eng.search(np.ones((5, 16), np.float32), "l2")
    np.testing.assert_array_equal(idx, -1)
    assert np.all(np.isnan(best))


@pytest.mark.parametrize("k", [64, 300])
def test_sharded_keys_min_equals_full(eng, k):
    """Row sharding with global offsets + MIN over keys == unsharded search (the
    multi-GPU all-reduce contract)."""
    rng = np.random.default_rng(9)
    g = rng.standard_normal((5000, k)).astype(np.float32)
    q = rng.standard_normal((700, k)).astype(np.float32)
    for metric in ("l2", "cosine"):
        eng.set_gallery(g)
        full = eng.search_keys(q, metric)
        parts = []
        for lo, hi in [(0, 1700), (1700, 3333), (3333, 5000)]:
            eng.set_gallery(g[lo:hi], global_offset=lo)
            parts.append(eng.search_keys(q, metric))
        np.testing.assert_array_equal(np.minimum.reduce(parts), full)


@pytest.mark.parametrize("n,k", [(200_000, 128), (100_000, 512)])
def test_planted_nearest_neighbour(eng, n, k):
    """Probes = gallery rows + small noise: the argmin identity is exact."""
    rng = np.random.default_rng(1)
    b = 4096
    g = (rng.standard_normal((n, k)) * orc.synth_spectrum(k)).astype(np.float32)
    t = rng.integers(0, n, b)
    q = (g[t] + rng.standard_normal((b, k)).astype(np.float32) * 2.0).astype(np.float32)
    eng.set_gallery(g)
    idx, d = eng.search(q, "l2")
    np.testing.assert_array_equal(idx, t)
    d_ref = ((q.astype(np.float64) - g[t]) ** 2).sum(1)
    np.testing.assert_allclose(d, d_ref, rtol=1e-4)
    idx_c, _ = eng.search(q, "cosine")
    np.testing.assert_array_equal(idx_c, t)
