"""k > 512: projection and gallery search at any feature width.

The reference's train-v5.py fits every person at full rank (n_components = face count,
/root/reference/train-v5.py:539-545) — its own faces/lock_version/shun holds 601 crops —
and its scanner projects and cosine-searches those models at whatever k they have
(scan-template-v4.py:265-287).  The engine pads k > 512 to a multiple of 128 and runs the
wide kernels with the row length at run time (ef_search_wide.hip KP = 0); everything is
checked against the fp64 oracle with the same tolerances as the k <= 512 tests."""
import numpy as np
import pytest

from oracle import eigenface_oracle as orc
from test_gpu_search import _check_cos as _cos_check, _check_l2

pytestmark = pytest.mark.gpu

WIDE_K = [513, 601, 1024]


@pytest.fixture(params=[0, 1, 2], ids=["fp32", "split16", "split32"])
def scan(eng, request):
    eng.set_option("search_split_bf16", request.param)
    yield eng
    eng.set_option("search_split_bf16", 0)


@pytest.mark.parametrize("k", WIDE_K)
@pytest.mark.parametrize("n,b", [(1, 3), (601, 601), (5003, 1100)])
def test_search_wide_k_vs_oracle(scan, k, n, b):
    rng = np.random.default_rng(k * 7 + n)
    g = rng.standard_normal((n, k)).astype(np.float32)
    q = rng.standard_normal((b, k)).astype(np.float32)
    scan.set_gallery(g)
    idx, best = scan.search(q, "l2")
    _check_l2(q, g, idx, best)
    idx, best = scan.search(q, "cosine")
    _cos_check(q, g, idx, best)


@pytest.mark.parametrize("k", WIDE_K)
def test_search_wide_k_keys_equal_across_scans(eng, k):
    """The split-bf16 scans resolve to the fp32 scan's keys bit for bit (planted + random
    probes, a blocked XCD deal at b = 2048, duplicates for the lowest-index rule)."""
    rng = np.random.default_rng(k)
    n, b = 7001, 2048
    g = rng.standard_normal((n, k)).astype(np.float32)
    g[4000] = g[17]
    t = rng.integers(0, n, b)
    q = (g[t] + 0.05 * rng.standard_normal((b, k))).astype(np.float32)
    q[: b // 4] = rng.standard_normal((b // 4, k))
    q[b // 4] = g[17]
    eng.set_gallery(g)
    out = {}
    for opt in (0, 1, 2):
        eng.set_option("search_split_bf16", opt)
        out[opt] = {m: eng.search_keys(q, m) for m in ("l2", "cosine")}
    eng.set_option("search_split_bf16", 0)
    for m in ("l2", "cosine"):
        np.testing.assert_array_equal(out[1][m], out[0][m])
        np.testing.assert_array_equal(out[2][m], out[0][m])
    idx, _ = eng.search(q, "l2")
    np.testing.assert_array_equal(idx[b // 4 + 1:], t[b // 4 + 1:])
    assert idx[b // 4] == 17


@pytest.mark.parametrize("k", [513, 1024])
def test_sharded_offsets_wide_k(eng, k):
    """Row shards with global offsets, MIN over keys == the unsharded search."""
    rng = np.random.default_rng(k + 3)
    g = rng.standard_normal((3000, k)).astype(np.float32)
    q = rng.standard_normal((300, k)).astype(np.float32)
    for metric in ("l2", "cosine"):
        eng.set_gallery(g)
        full = eng.search_keys(q, metric)
        parts = []
        for lo, hi in [(0, 1111), (1111, 3000)]:
            eng.set_gallery(g[lo:hi], global_offset=lo)
            parts.append(eng.search_keys(q, metric))
        np.testing.assert_array_equal(np.minimum.reduce(parts), full)


@pytest.mark.parametrize("k", WIDE_K)
@pytest.mark.parametrize("b", [1, 300])
def test_project_wide_k(eng, k, b):
    d = 4096
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
    # bf16 model at the same width: the stated config-5 tolerance
    eng.set_model(mu, w, precision="bf16")
    f16 = eng.project(p)
    a = np.abs(p.astype(np.float64) - np.rint(mu))
    bound16 = 2.0 ** -8 * (a @ np.abs(w.astype(np.float64))) + 2e-6 * bound + 1e-5
    assert np.all(np.abs(f16 - ref) <= bound16)


@pytest.mark.parametrize("k", [601, 1024])
def test_recognize_fused_wide_k(eng, k):
    """Fused projection + search at k > 512 (the full-rank train-v5 shape): planted
    probes recover their rows, and the keys equal project-then-search."""
    rng = np.random.default_rng(k + 11)
    d = 4096
    mu = rng.uniform(60, 200, d).astype(np.float32)
    w = np.linalg.qr(rng.standard_normal((d, k)))[0].astype(np.float32)
    gal = rng.integers(0, 256, (2500, d), dtype=np.uint8)
    eng.set_model(mu, w)
    eng.set_gallery(eng.project(gal))
    probes = np.clip(gal[::5].astype(np.int32) + rng.integers(-3, 4, (500, d)), 0, 255).astype(np.uint8)
    for metric in ("l2", "cosine"):
        idx, best = eng.recognize(probes, metric)
        np.testing.assert_array_equal(idx, np.arange(0, 2500, 5))
        idx2, best2 = eng.search(eng.project(probes), metric)
        np.testing.assert_array_equal(idx2, idx)
        np.testing.assert_array_equal(best2, best)


def test_probe_batch_pieces_at_huge_k(eng):
    """bpad x kp x 4 >= 2^31: the engine searches the batch in pieces of whole probe tiles
    (32-bit probe-row offsets in the kernels).  k = 65536, 8200 probes = two pieces."""
    k, n, b = 65536, 40, 8200
    rng = np.random.default_rng(77)
    g = rng.standard_normal((n, k), dtype=np.float32)
    t = rng.integers(0, n, b)
    q = g[t].copy()
    q += np.float32(0.5) * rng.standard_normal((b, k), dtype=np.float32)
    eng.set_gallery(g)
    idx, best = eng.search(q, "l2")
    np.testing.assert_array_equal(idx, t)
    d_ref = np.empty(b)
    for i in range(0, b, 512):
        e = q[i:i + 512].astype(np.float64) - g[t[i:i + 512]]
        d_ref[i:i + 512] = np.einsum("ij,ij->i", e, e)
    np.testing.assert_allclose(best, d_ref, rtol=1e-4)
    idx_c, _ = eng.search(q, "cosine")
    np.testing.assert_array_equal(idx_c, t)
