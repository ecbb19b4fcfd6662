"""Split-bf16 gallery scan (EF_OPT_SEARCH_SPLIT_BF16): the scan runs on bf16 MFMA with
(hi, lo) operands and a widened error bound; the winner is fp64-resolved exactly as on the
fp32 scan.  Both paths return the fp64 argmin/argmax with lowest-index ties, so their keys
must be identical bit for bit, and equal the fp64 oracle wherever the oracle's own
runner-up gap is clear."""
import numpy as np
import pytest

from conftest import golden
from oracle import eigenface_oracle as orc

pytestmark = pytest.mark.gpu


@pytest.fixture
def split(eng):
    eng.set_option("search_split_bf16", 1)
    yield eng
    eng.set_option("search_split_bf16", 0)


def _keys_both(eng, g, q, metric, offset=0):
    eng.set_option("search_split_bf16", 0)
    eng.set_gallery(g, global_offset=offset)
    k32 = eng.search_keys(q, metric)
    eng.set_option("search_split_bf16", 1)
    k3 = eng.search_keys(q, metric)  # the split copy is built on this first split search
    return k32, k3


def test_option_roundtrip(split):
    assert split.get_option("search_split_bf16") == 1


@pytest.mark.parametrize("k", [8, 16, 50, 64, 96, 128, 200])
@pytest.mark.parametrize("n,b", [(1, 3), (33, 257), (3001, 300)])
def test_split_keys_equal_fp32_random(split, k, n, b):
    rng = np.random.default_rng(k * 7 + n)
    g = rng.standard_normal((n, k)).astype(np.float32)
    q = rng.standard_normal((b, k)).astype(np.float32)
    for metric in ("l2", "cosine"):
        k32, k3 = _keys_both(split, g, q, metric)
        np.testing.assert_array_equal(k3, k32)


@pytest.mark.parametrize("k", [64, 128])
def test_split_matches_oracle(split, k):
    rng = np.random.default_rng(k)
    g = rng.standard_normal((20000, k)).astype(np.float32)
    q = rng.standard_normal((1000, k)).astype(np.float32)
    split.set_gallery(g)
    idx, best = split.search(q, "l2")
    ref_idx, ref_d = orc.l2_argmin(q, g)
    g64, q64 = g.astype(np.float64), q.astype(np.float64)
    dd = (q64**2).sum(1)[:, None] + (g64**2).sum(1)[None, :] - 2.0 * q64 @ g64.T
    s = np.partition(dd, 1, axis=1)[:, :2]
    clear = (s[:, 1] - s[:, 0]) > 1e-9 * (q64**2).sum(1)
    assert clear.mean() > 0.99
    np.testing.assert_array_equal(idx[clear], ref_idx[clear])
    d_gpu = ((q64 - g64[idx]) ** 2).sum(1)
    np.testing.assert_allclose(best, d_gpu.astype(np.float32), rtol=1e-6)
    idx_c, _ = split.search(q, "cosine")
    ref_c, _ = orc.cosine_argmax(q, g)
    srt = np.sort(orc.cosine_scores(q, g), axis=1)
    clear_c = (srt[:, -1] - srt[:, -2]) > 1e-9
    np.testing.assert_array_equal(idx_c[clear_c], ref_c[clear_c])


@pytest.mark.parametrize("k", [32, 128])
def test_split_near_ties_below_bf16_resolution(split, k):
    """Rows whose distances to the probe differ by ~1e-6 relative (far below the split
    scan's ~1e-4 resolution, far above fp64's): the exact winner is the later row."""
    rng = np.random.default_rng(11 + k)
    n, b = 5000, 256
    g = rng.standard_normal((n, k)).astype(np.float32)
    q = rng.standard_normal((b, k)).astype(np.float32)
    for i in range(b):
        d = rng.standard_normal(k).astype(np.float32) * 0.5
        lo, hi = rng.choice(n, 2, replace=False)
        lo, hi = min(lo, hi), max(lo, hi)
        g[lo] = q[i] + d
        g[hi] = q[i] + d * np.float32(1 - 2e-6)  # closer by ~4e-6 relative
    # exact fp64 winners (the planted pairs can collide with each other's rows)
    want = orc.l2_argmin(q, g)[0]
    k32, k3 = _keys_both(split, g, q, "l2")
    np.testing.assert_array_equal(k3, k32)
    idx = (k3 & 0xFFFFFFFF).astype(np.int64)
    np.testing.assert_array_equal(idx, want)


def test_split_duplicates_and_ties_golden(split):
    g = np.random.default_rng(5).standard_normal((1000, 32)).astype(np.float32)
    g[700] = g[5]
    g[999] = g[5]
    g[300] = g[64]
    q = np.stack([g[5], g[999], g[64], g[300]])
    split.set_gallery(g)
    idx, d = split.search(q, "l2")
    np.testing.assert_array_equal(idx, [5, 5, 64, 64])
    np.testing.assert_array_equal(d, [0, 0, 0, 0])
    t = golden("ties.npz")
    split.set_gallery(t["gallery"].astype(np.float32))
    idx, sim = split.search(t["probes"].astype(np.float32), "cosine")
    np.testing.assert_array_equal(idx, t["idx"])
    np.testing.assert_allclose(sim, t["sim"], atol=1e-6)


def test_split_sharded_offsets(split):
    rng = np.random.default_rng(9)
    g = rng.standard_normal((5000, 64)).astype(np.float32)
    q = rng.standard_normal((700, 64)).astype(np.float32)
    for metric in ("l2", "cosine"):
        split.set_gallery(g)
        full = split.search_keys(q, metric)
        parts = []
        for lo, hi in [(0, 1700), (1700, 3333), (3333, 5000)]:
            split.set_gallery(g[lo:hi], global_offset=lo)
            parts.append(split.search_keys(q, metric))
        np.testing.assert_array_equal(np.minimum.reduce(parts), full)


def test_split_planted_large(split):
    """The C3 shape at 200k rows: planted probes (gallery row + noise) are exact."""
    rng = np.random.default_rng(1)
    n, k, b = 200_000, 128, 4096
    g = (rng.standard_normal((n, k)) * orc.synth_spectrum(k)).astype(np.float32)
    t = rng.integers(0, n, b)
    q = (g[t] + rng.standard_normal((b, k)).astype(np.float32) * 2.0).astype(np.float32)
    k32, k3 = _keys_both(split, g, q, "l2")
    np.testing.assert_array_equal(k3, k32)
    np.testing.assert_array_equal((k3 & 0xFFFFFFFF).astype(np.int64), t)
    k32c, k3c = _keys_both(split, g, q, "cosine")
    np.testing.assert_array_equal(k3c, k32c)


@pytest.mark.parametrize("k", [256, 300, 512])
def test_split_wide_keys_equal_fp32(split, k):
    """k > 128: the wide kernel streams split probes and split gallery slices."""
    rng = np.random.default_rng(3 + k)
    g = rng.standard_normal((3001, k)).astype(np.float32)
    q = rng.standard_normal((1100, k)).astype(np.float32)
    for metric in ("l2", "cosine"):
        k32, k3 = _keys_both(split, g, q, metric)
        np.testing.assert_array_equal(k3, k32)


@pytest.mark.parametrize("k", [256, 512])
def test_split_wide_near_ties(split, k):
    rng = np.random.default_rng(17 + k)
    n, b = 4000, 300
    g = rng.standard_normal((n, k)).astype(np.float32)
    q = rng.standard_normal((b, k)).astype(np.float32)
    for i in range(b):
        d = rng.standard_normal(k).astype(np.float32) * 0.5
        lo, hi = sorted(rng.choice(n, 2, replace=False))
        g[lo] = q[i] + d
        g[hi] = q[i] + d * np.float32(1 - 2e-6)
    want = orc.l2_argmin(q, g)[0]
    k32, k3 = _keys_both(split, g, q, "l2")
    np.testing.assert_array_equal(k3, k32)
    np.testing.assert_array_equal((k3 & 0xFFFFFFFF).astype(np.int64), want)


@pytest.mark.parametrize("b", [1024, 2048, 4096])
def test_split_wide_xcd_deal(split, b):
    """Batches of >= 8 split probe tiles take the blocked (4 probe tiles x cblk chunks)
    XCD deal of the 256 x 256 split wide kernel; ragged last gallery tile."""
    rng = np.random.default_rng(b)
    g = rng.standard_normal((5003, 512)).astype(np.float32)
    q = rng.standard_normal((b, 512)).astype(np.float32)
    for metric in ("l2", "cosine"):
        k32, k3 = _keys_both(split, g, q, metric)
        np.testing.assert_array_equal(k3, k32)


@pytest.mark.parametrize("k", [100, 128, 256, 300, 512])
def test_split_kernel_shapes_agree(split, k):
    """k in (64, 128] and the wide scans (k > 128): the default 16x16x32 split kernels
    (search16_kernel, search_wide16_kernel) and the 32x32x16 ones (option 2:
    search_kernel<S3>, search_wide3_kernel) return the fp32 scan's keys, on random probes
    and on sub-bf16 near-ties."""
    rng = np.random.default_rng(k + 5)
    n, b = 7001, 700
    g = rng.standard_normal((n, k)).astype(np.float32)
    q = rng.standard_normal((b, k)).astype(np.float32)
    for i in range(0, b, 2):
        d = rng.standard_normal(k).astype(np.float32) * 0.5
        lo, hi = sorted(rng.choice(n, 2, replace=False))
        g[lo] = q[i] + d
        g[hi] = q[i] + d * np.float32(1 - 2e-6)
    for metric in ("l2", "cosine"):
        k32, k16 = _keys_both(split, g, q, metric)
        split.set_option("search_split_bf16", 2)
        k3232 = split.search_keys(q, metric)
        np.testing.assert_array_equal(k16, k32)
        np.testing.assert_array_equal(k3232, k32)
    assert split.get_option("search_split_bf16") == 2


@pytest.mark.parametrize("k", [64, 128, 512])
def test_candidate_overflow_cluster(split, k):
    """A cluster of 200 rows within 1e-6 of each other around the probes: every row of the
    cluster is inside the scan's bound, more than the 32 kept candidates, so the resolve
    pass re-scores the whole gallery in fp64 — fp32 and split scans both return the fp64
    argmin (np.argmin semantics)."""
    rng = np.random.default_rng(k + 99)
    n, b = 3000, 64
    g = rng.standard_normal((n, k)).astype(np.float32)
    base = rng.standard_normal(k).astype(np.float32)
    g[100:300] = base + (rng.standard_normal((200, k)) * 1e-6).astype(np.float32)
    q = (base + rng.standard_normal((b, k)).astype(np.float32) * 0.01).astype(np.float32)
    want = orc.l2_argmin(q, g)[0]
    k32, k3 = _keys_both(split, g, q, "l2")
    np.testing.assert_array_equal((k32 & 0xFFFFFFFF).astype(np.int64), want)
    np.testing.assert_array_equal(k3, k32)


@pytest.mark.parametrize("k", [64, 128, 512])
def test_split_match_records_equal_fp32(split, k):
    """The exact cross-shard merge consumes match records (fp64 score, tie scale, key):
    the split scan's records equal the fp32 scan's field for field, per shard, and the
    merged keys equal the single-gallery keys."""
    rng = np.random.default_rng(k + 2)
    g = rng.standard_normal((4000, k)).astype(np.float32)
    q = rng.standard_normal((600, k)).astype(np.float32)
    for metric in ("l2", "cosine"):
        recs = {}
        for opt in (0, 1):
            split.set_option("search_split_bf16", opt)
            parts = []
            for lo, hi in [(0, 1500), (1500, 4000)]:
                split.set_gallery(g[lo:hi], global_offset=lo)
                parts.append(split.search_matches(q, metric))
            recs[opt] = parts
            from eigenface import merge_matches_host
            merged = merge_matches_host(np.concatenate(parts), len(q))
            split.set_gallery(g)
            np.testing.assert_array_equal(merged, split.search_keys(q, metric))
        for a, b in zip(recs[0], recs[1]):
            for f in ("score", "scale", "key"):
                np.testing.assert_array_equal(a[f], b[f])


# ---- the single-bf16 screen (option 3, k > 128): one bf16 MFMA per product, a bound 2^8
# times wider than the split scan's; probes whose best rows are within it are collected and
# fp64-resolved, so the keys still equal the fp32 scan's bit for bit.

def _keys_screen(eng, g, q, metric, offset=0):
    eng.set_option("search_split_bf16", 0)
    eng.set_gallery(g, global_offset=offset)
    k32 = eng.search_keys(q, metric)
    eng.set_option("search_split_bf16", 3)
    try:
        k1 = eng.search_keys(q, metric)  # the single-bf16 copy is built on this first search
    finally:
        eng.set_option("search_split_bf16", 0)
    return k32, k1


def test_screen_option_roundtrip(eng):
    eng.set_option("search_split_bf16", 3)
    try:
        assert eng.get_option("search_split_bf16") == 3
    finally:
        eng.set_option("search_split_bf16", 0)
    with pytest.raises(Exception):
        eng.set_option("search_split_bf16", 4)


@pytest.mark.parametrize("k", [256, 300, 512, 640, 1024])
def test_screen_keys_equal_fp32(eng, k):
    """Random Gaussian rows: the best two rows of a probe are often within the bf16 bound
    (many probes take the collect pass, some overflow its 32 candidates and are re-scored
    over the whole gallery) — keys identical to the fp32 scan either way."""
    rng = np.random.default_rng(31 + k)
    g = rng.standard_normal((3001, k)).astype(np.float32)
    q = rng.standard_normal((1100, k)).astype(np.float32)
    for metric in ("l2", "cosine"):
        k32, k1 = _keys_screen(eng, g, q, metric)
        np.testing.assert_array_equal(k1, k32)


@pytest.mark.parametrize("k", [256, 512])
def test_screen_near_ties_and_planted(eng, k):
    """Sub-bf16 near-ties (the later row closer by ~4e-6 relative) and planted probes in
    one batch: exact fp64 winners."""
    rng = np.random.default_rng(71 + k)
    n, b = 6000, 512
    g = rng.standard_normal((n, k)).astype(np.float32)
    q = rng.standard_normal((b, k)).astype(np.float32)
    for i in range(0, b, 2):
        d = rng.standard_normal(k).astype(np.float32) * 0.5
        lo, hi = sorted(rng.choice(n, 2, replace=False))
        g[lo] = q[i] + d
        g[hi] = q[i] + d * np.float32(1 - 2e-6)
    t = rng.integers(0, n, b)
    q[1::2] = g[t[1::2]] + rng.standard_normal((b // 2, k)).astype(np.float32) * 0.1
    want = orc.l2_argmin(q, g)[0]
    k32, k1 = _keys_screen(eng, g, q, "l2")
    np.testing.assert_array_equal(k1, k32)
    np.testing.assert_array_equal((k1 & 0xFFFFFFFF).astype(np.int64), want)


@pytest.mark.parametrize("b", [1024, 4096])
def test_screen_xcd_deal_and_ragged_tile(eng, b):
    rng = np.random.default_rng(b + 3)
    g = rng.standard_normal((5003, 512)).astype(np.float32)
    t = rng.integers(0, 5003, b)
    q = (g[t] + rng.standard_normal((b, 512)).astype(np.float32) * 0.3).astype(np.float32)
    for metric in ("l2", "cosine"):
        k32, k1 = _keys_screen(eng, g, q, metric)
        np.testing.assert_array_equal(k1, k32)
        np.testing.assert_array_equal((k1 & 0xFFFFFFFF).astype(np.int64), t)


def test_screen_cluster_overflow_and_records(eng):
    """A 200-row cluster inside 1e-6 (candidate overflow -> whole-gallery fp64 re-score) and
    the match records of two shards: field for field equal to the fp32 scan's."""
    rng = np.random.default_rng(515)
    k, n, b = 512, 3000, 64
    g = rng.standard_normal((n, k)).astype(np.float32)
    base = rng.standard_normal(k).astype(np.float32)
    g[100:300] = base + (rng.standard_normal((200, k)) * 1e-6).astype(np.float32)
    q = (base + rng.standard_normal((b, k)).astype(np.float32) * 0.01).astype(np.float32)
    k32, k1 = _keys_screen(eng, g, q, "l2")
    np.testing.assert_array_equal((k32 & 0xFFFFFFFF).astype(np.int64), orc.l2_argmin(q, g)[0])
    np.testing.assert_array_equal(k1, k32)
    recs = {}
    for opt in (0, 3):
        eng.set_option("search_split_bf16", opt)
        try:
            recs[opt] = [None, None]
            for j, (lo, hi) in enumerate([(0, 1500), (1500, 3000)]):
                eng.set_gallery(g[lo:hi], global_offset=lo)
                recs[opt][j] = eng.search_matches(q, "cosine")
        finally:
            eng.set_option("search_split_bf16", 0)
    for a, c in zip(recs[0], recs[3]):
        for f in ("score", "scale", "key"):
            np.testing.assert_array_equal(a[f], c[f])
