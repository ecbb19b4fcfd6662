"""The N>1 path on CPU: world_size-2/3 gloo, row-sharded gallery, all-gather of the
per-rank fp64 match records + the library's exact merge (ef_matches_merge, host form) ==
unsharded arg-best with lowest-index ties — including winners in different shards whose
fp64 scores differ by less than one fp32 ulp.  The per-rank search here is the oracle
(the GPU kernel's records are checked on the GPU by tests/test_gpu_distributed.py)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _paths():
    import sys
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)


def _scores64(q, g, metric):
    q = np.asarray(q, np.float64)
    g = np.asarray(g, np.float64)
    if metric == "l2":
        return ((q[:, None, :] - g[None, :, :]) ** 2).sum(-1)
    qn = np.linalg.norm(q, axis=1)
    gn = np.linalg.norm(g, axis=1)
    dots = q @ g.T
    with np.errstate(invalid="ignore", divide="ignore"):
        sim = dots / (qn[:, None] * gn[None, :])
    sim[(qn[:, None] == 0) | (gn[None, :] == 0)] = 0.0
    return -sim


def _oracle_matches(q, g_local, lo, metric):
    """One shard's records by the single-engine rule: lowest index among rows whose fp64
    score is within 1e-12 * (|min| + scale) of the shard's minimum."""
    _paths()
    from eigenface.distributed import make_matches
    q = np.asarray(q)
    if len(g_local) == 0:
        return make_matches(np.full(len(q), np.inf), np.zeros(len(q)), np.zeros(len(q), np.int64))
    s = _scores64(q, g_local, metric)
    g64 = np.asarray(g_local, np.float64)
    scale = ((np.asarray(q, np.float64) ** 2).sum(1) + (g64 ** 2).sum(1).max()) if metric == "l2" \
        else np.ones(len(q))
    vmin = s.min(axis=1)
    tol = 1e-12 * (np.abs(vmin) + scale)
    idx = np.argmax(s <= (vmin + tol)[:, None], axis=1)
    return make_matches(s[np.arange(len(q)), idx], scale, idx + lo)


def _oracle_keys(q, g, metric):
    return _oracle_matches(q, g, 0, metric)["key"]


def _worker(rank, world, port, g, q, metric, out, merge="exact"):
    import sys
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from eigenface.distributed import ShardedGallery, shard_range
    lo, hi = shard_range(len(g), rank, world)
    sg = ShardedGallery(None, g[lo:hi], len(g), rank, world,
                        local_matches=lambda qq, m: _oracle_matches(qq, g[lo:hi], lo, m), merge=merge)
    keys = sg.search_keys(q, metric)
    out[rank] = keys.numpy().copy()
    dist.destroy_process_group()


@pytest.mark.parametrize("metric", ["l2", "cosine"])
@pytest.mark.parametrize("world", [2, 3])
def test_sharded_allreduce_matches_unsharded(metric, world):
    rng = np.random.default_rng(world)
    g = rng.standard_normal((1001, 24)).astype(np.float32)
    g[600] = g[17]          # duplicate across shards: lowest index must win
    g[999] = 3.0 * g[40]    # cosine tie across shards
    q = rng.standard_normal((64, 24)).astype(np.float32)
    q[0] = g[17]
    q[1] = g[40]
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    out = mgr.dict()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, g, q, metric, out)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    full = _oracle_keys(q, g, metric)
    for r in range(world):
        np.testing.assert_array_equal(out[r], full)
    from eigenface import decode_keys
    idx, _ = decode_keys(full, metric)
    assert idx[0] == 17
    if metric == "cosine":
        assert idx[1] == 40


def test_shard_range_partitions_rows():
    from eigenface.distributed import shard_range
    for n in (0, 1, 7, 1000, 1_000_000):
        for w in (1, 2, 3, 8):
            rs = [shard_range(n, r, w) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(w - 1))
            assert max(h - l for l, h in rs) - min(h - l for l, h in rs) <= 1


def test_pack_keys_matches_library_decoder():
    from eigenface import decode_keys
    from eigenface.distributed import pack_keys
    v = np.array([-2.5, -0.0, 0.0, 1e-20, 3.0, np.inf], np.float32)
    i = np.arange(6) + 100
    k = pack_keys(v, i)
    idx, best = decode_keys(k, "l2")
    np.testing.assert_array_equal(idx, i)
    np.testing.assert_array_equal(best, np.where(v == 0, 0.0, v).astype(np.float32))
    assert np.all(np.diff(k[[0, 2, 3, 4, 5]]) > 0)


def _proj_worker(rank, world, port, g, P, mean, W, metric, out):
    import sys
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from eigenface.distributed import ShardedGallery, shard_range
    from oracle import eigenface_oracle as orc
    lo, hi = shard_range(len(g), rank, world)
    seen = []

    def proj(p, out=None):  # records which probe rows this rank projected
        seen.append(len(p))
        return torch.from_numpy(orc.project(p.numpy(), mean, W).astype(np.float32))

    sg = ShardedGallery(None, g[lo:hi], len(g), rank, world, local_project=proj,
                        local_matches=lambda qq, m: _oracle_matches(qq.numpy(), g[lo:hi], lo, m))
    keys = sg.recognize_keys(torch.from_numpy(P), metric)
    out[rank] = (keys.numpy().copy(), sum(seen))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,b", [(2, 64), (3, 67), (4, 5)])
def test_sharded_projection_allgather_matches_unsharded(world, b):
    """world > 1: each rank projects ceil(B/world) probe rows, the features are
    all-gathered, then the sharded search + all-reduce(MIN) equals the unsharded result."""
    import sys
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    from oracle import eigenface_oracle as orc
    rng = np.random.default_rng(b)
    d, k = 64, 12
    W = np.linalg.qr(rng.standard_normal((d, k)))[0].astype(np.float32)
    mean = rng.uniform(60, 200, d).astype(np.float32)
    g = rng.standard_normal((301, k)).astype(np.float32) * 30
    P = rng.integers(0, 256, (b, d)).astype(np.uint8)
    ctx = mp.get_context("spawn")
    out = ctx.Manager().dict()
    port = _free_port()
    procs = [ctx.Process(target=_proj_worker, args=(r, world, port, g, P, mean, W, "l2", out))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    q = orc.project(P, mean, W).astype(np.float32)
    full = _oracle_keys(q, g, "l2")
    c = (b + world - 1) // world
    for r in range(world):
        np.testing.assert_array_equal(out[r][0], full)
        assert out[r][1] == max(0, min(b, (r + 1) * c) - min(b, r * c))


def sub_ulp_case(k=24, n=400, seed=0):
    """Gallery + probes where the true winner sits in a later shard and beats a row of an
    earlier shard by ~1e-9 relative — below fp32 resolution of the score, far above the
    1e-12 tie tolerance.  A MIN over packed fp32 keys would return the earlier row.
    Returns (g, q, rows_a, rows_b, metric_of_probe)."""
    rng = np.random.default_rng(seed)
    g = (rng.standard_normal((n, k)) * 4.0).astype(np.float32)
    q = np.zeros((4, k), np.float32)
    # L2 probes 0, 1: g_a = q + 0.5 e0 (d^2 = 0.25); g_b = q + x e1 + y e2 with
    # x = 0.5 - 2^-24, x^2 + y^2 = 0.25 - 1e-9 (both round to the same fp32 distance)
    x = np.float32(0.5) - np.float32(2.0 ** -24)
    y = np.float32(np.sqrt(0.25 - 1e-9 - float(x) ** 2))
    rows_a, rows_b = [], []
    for j, (ra, rb) in enumerate([(10, 390), (150, 260)]):
        base = (np.rint(rng.standard_normal(k) * 20) / 64).astype(np.float32)
        base[:3] = 0  # the offsets below are then exact in fp32
        q[j] = base
        g[ra] = base
        g[ra, 0] += np.float32(0.5)
        g[rb] = base
        g[rb, 1] += x
        g[rb, 2] += y
        rows_a.append(ra)
        rows_b.append(rb)
    # cosine probes 2, 3: q = e0; g_a = (1, a), g_b = (1, b) with 1/sqrt(1+b^2) - 1/sqrt(1+a^2) ~ 1e-9
    a = np.float32(1e-3)
    bb = np.float32(np.sqrt(float(a) ** 2 - 2e-9))
    for j, (ra, rb), ax in zip((2, 3), [(20, 380), (100, 200)], (0, 5)):
        q[j] = 0
        q[j, ax] = 1
        g[ra] = 0
        g[ra, ax], g[ra, ax + 3] = 1, a
        g[rb] = 0
        g[rb, ax], g[rb, ax + 4] = 1, bb
        rows_a.append(ra)
        rows_b.append(rb)
    return g, q, rows_a, rows_b


def test_sub_ulp_case_is_a_real_fp32_tie():
    g, q, ra, rb = sub_ulp_case()
    s_l2 = _scores64(q[:2], g, "l2")
    s_cos = _scores64(q[2:], g, "cosine")
    for s, a, b in ((s_l2, ra[:2], rb[:2]), (s_cos, ra[2:], rb[2:])):
        for i in range(2):
            va, vb = s[i, a[i]], s[i, b[i]]
            assert vb < va and (va - vb) / abs(va) > 1e-10        # b is strictly better in fp64
            assert np.float32(va) == np.float32(vb)                 # ... but ties in fp32
            assert np.argmin(s[i]) == b[i]
    # the fp32 key MIN across shards would pick the earlier row
    from eigenface.distributed import pack_keys
    ka = pack_keys(np.float32(s_l2[0, ra[0]]), ra[0])
    kb = pack_keys(np.float32(s_l2[0, rb[0]]), rb[0])
    assert min(ka, kb) == ka


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_merge_is_fp64_exact_across_shards(world):
    g, q, ra, rb = sub_ulp_case()
    ctx = mp.get_context("spawn")
    out = ctx.Manager().dict()
    res = {}
    for metric, qs in (("l2", q[:2]), ("cosine", q[2:])):
        port = _free_port()
        procs = [ctx.Process(target=_worker, args=(r, world, port, g, qs, metric, out)) for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(120)
            assert p.exitcode == 0
        res[metric] = [out[r] for r in range(world)]
    from eigenface import decode_keys
    for metric, want in (("l2", rb[:2]), ("cosine", rb[2:])):
        for r in range(world):
            idx, _ = decode_keys(res[metric][r], metric)
            np.testing.assert_array_equal(idx, want)


@pytest.mark.parametrize("world", [2, 3])
def test_min_allreduce_merge(world):
    """merge="min" (the north star's single all-reduce(MIN) of packed keys): equal to the
    exact merge on duplicates and cosine ties across shards; on the sub-ulp case (winners
    of different shards tied in fp32, not in fp64) it keeps the lower index, where the
    exact merge returns the fp64 winner."""
    rng = np.random.default_rng(40 + world)
    g = rng.standard_normal((1001, 24)).astype(np.float32)
    g[600] = g[17]
    g[999] = 3.0 * g[40]
    q = rng.standard_normal((64, 24)).astype(np.float32)
    q[0] = g[17]
    q[1] = g[40]
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    for metric in ("l2", "cosine"):
        out = mgr.dict()
        port = _free_port()
        procs = [ctx.Process(target=_worker, args=(r, world, port, g, q, metric, out, "min")) for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(120)
            assert p.exitcode == 0
        full = _oracle_keys(q, g, metric)
        for r in range(world):
            np.testing.assert_array_equal(out[r], full)
    gs, qs, ra, rb = sub_ulp_case()
    from eigenface import decode_keys
    from eigenface.distributed import shard_range
    shard = [next(r for r in range(world) if shard_range(len(gs), r, world)[0] <= i < shard_range(len(gs), r, world)[1])
             for i in range(len(gs))]
    # across shards the fp32 tie keeps the lower index; inside one shard its fp64 resolution holds
    want_all = [a if shard[a] != shard[b] else b for a, b in zip(ra, rb)]
    for metric, qq, want in (("l2", qs[:2], want_all[:2]), ("cosine", qs[2:], want_all[2:])):
        out = mgr.dict()
        port = _free_port()
        procs = [ctx.Process(target=_worker, args=(r, world, port, gs, qq, metric, out, "min")) for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(120)
            assert p.exitcode == 0
        for r in range(world):
            idx, _ = decode_keys(out[r], metric)
            np.testing.assert_array_equal(idx, want)


def test_merge_mode_is_checked():
    _paths()
    from eigenface.distributed import ShardedGallery
    with pytest.raises(ValueError):
        ShardedGallery(None, None, 10, 0, 1, merge="sum")


# ------------------------------------------------------------- sample-sharded fit
def _np_pieces(x):
    """The exact integer pieces of include/eigenface.h ef_fit_shard_stats, in numpy."""
    xi = np.asarray(x, np.int64)
    xs = xi - 128
    return xi.sum(0), (xi * xi).sum(0), xs.T @ xs


def _np_fit_from_pieces(s1, s2, cr, n, k, standardize):
    """ef_fit_from_stats's arithmetic restated (the covariance from exact integers,
    oracle.top_eigh): what the sum over ranks must reproduce."""
    _paths()
    from eigenface import FitResult
    from oracle import eigenface_oracle as orc
    s1, s2, cr = (np.asarray(a, np.int64) for a in (s1, s2, cr))
    mean = s1 / n
    var = (n * s2 - s1 * s1) / float(n) ** 2
    scale = np.where(var > 0, np.sqrt(var), 1.0) if standardize else np.ones_like(mean)
    c = s1 - 128 * n
    C = (n * cr.astype(np.float64) - np.outer(c, c).astype(np.float64)) / (n * (n - 1.0))
    C /= np.outer(scale, scale)
    lam, vt = orc.top_eigh(C.copy(), k)
    return FitResult(mean, var, scale, vt, lam, None, float(np.trace(C)), k, 0)


def _fit_worker(rank, world, port, x, k, standardize, out):
    import sys
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from eigenface.distributed import shard_range, sharded_fit
    lo, hi = shard_range(len(x), rank, world)
    xl = x[lo:hi]

    def transform(rows, res, stdz):
        z = (np.asarray(rows, np.float64) - res.mean) / res.scale
        return z @ res.components.T
    res = sharded_fit(None, xl, k, standardize, stats_fn=_np_pieces, fit_fn=_np_fit_from_pieces,
                      transform_fn=transform)
    out[rank] = (res.eigenvalues.copy(), res.components.copy(), res.projection.copy(), res.mean.copy())
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_fit_pieces_allreduce(world):
    """distributed.sharded_fit on gloo (world 2 / 3, uneven shards): n_total and the summed
    integer pieces reach every rank, every rank fits the same model, and the per-rank
    projections stack to the projection of the whole set — equal to the fit from the
    pieces of all rows at once (and to the oracle's covariance-path PCA)."""
    _paths()
    from oracle import eigenface_oracle as orc
    x, _ = orc.synth_faces(401, 8, r=20, seed=world)  # n = 401 >= d = 64
    k = 10
    ref = _np_fit_from_pieces(*_np_pieces(x), len(x), k, True)
    o = orc.pca_cov_fit(x, k, standardize=True)
    np.testing.assert_allclose(ref.eigenvalues, o["explained_variance_"], rtol=1e-9)
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_fit_worker, args=(world, _free_port(), x, k, True, out), nprocs=world, join=True)
    for r in range(world):
        lam, comps, proj, mean = out[r]
        np.testing.assert_array_equal(lam, ref.eigenvalues)
        np.testing.assert_array_equal(comps, ref.components)
        np.testing.assert_array_equal(mean, ref.mean)
    proj = np.concatenate([out[r][2] for r in range(world)])
    z = (x.astype(np.float64) - ref.mean) / ref.scale
    np.testing.assert_allclose(proj, z @ ref.components.T, atol=1e-9)


def test_fit_stats_allreduce_routes_host_pieces_for_device_backends(monkeypatch):
    """with a device-collective backend (RCCL, "nccl" on ROCm) the host
    pieces of a host X_local must travel through the device instead of being handed to
    all_reduce as CPU tensors (which RCCL rejects), and come back summed; with gloo, device
    pieces reduce through host copies.  One predicate (_device_collectives) decides for
    the gallery and the fit.  Backend and all_reduce are mocked (x2 = a two-rank sum)."""
    _paths()
    import torch
    import torch.distributed as dist
    from eigenface import distributed as D
    seen = []

    def fake_all_reduce(t, group=None, op=None):
        seen.append(t.device.type)
        t.mul_(2)

    monkeypatch.setattr(dist, "all_reduce", fake_all_reduce)
    for backend, expect in (("nccl", True), ("gloo", False)):
        monkeypatch.setattr(dist, "get_backend", lambda group=None, b=backend: b)
        assert D._device_collectives() is expect
        seen.clear()
        sx = np.arange(128, dtype=np.int64)
        gram = np.arange(128 * 128, dtype=np.int64).reshape(128, 128)
        out = D.allreduce_fit_stats([sx.copy(), gram.copy()], device="cpu")
        np.testing.assert_array_equal(out[0].numpy(), 2 * sx)
        iu = np.triu_indices(2)
        blocks = out[1].numpy().reshape(2, 64, 2, 64).transpose(0, 2, 1, 3)
        ref = gram.reshape(2, 64, 2, 64).transpose(0, 2, 1, 3)
        for a, b in zip(*iu):  # the upper 64-blocks travel (and come back summed)
            np.testing.assert_array_equal(blocks[a, b], 2 * ref[a, b])
        np.testing.assert_array_equal(blocks[1, 0], ref[1, 0])  # the lower block stays local
        assert seen == ["cpu", "cpu"]
