"""The N>1 path on CPU: world_size-2 gloo, row-sharded gallery, all-reduce(MIN) over
packed keys == unsharded arg-best with lowest-index ties.  The per-rank search here is
the oracle (the GPU kernel's key format is checked separately against the library's
decoder and on the GPU by test_gpu_search.test_sharded_keys_min_equals_full)."""
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


def _oracle_keys(q, g_local, lo, metric):
    import sys
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    from eigenface.distributed import pack_keys
    from oracle import eigenface_oracle as orc
    if len(g_local) == 0:
        return np.full(len(q), (1 << 63) - 1, dtype=np.int64)
    if metric == "l2":
        idx, d2 = orc.l2_argmin(q, g_local)
        return pack_keys(d2.astype(np.float32), idx + lo)
    idx, s = orc.cosine_argmax(q, g_local)
    return pack_keys(-s.astype(np.float32), idx + lo)


def _worker(rank, world, port, g, q, metric, out):
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
                        local_search=lambda qq, m, keys=None: _oracle_keys(qq, g[lo:hi], lo, m))
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
    full = _oracle_keys(q, g, 0, metric)
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
                        local_search=lambda qq, m, keys=None: _oracle_keys(qq.numpy(), g[lo:hi], lo, m))
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
    full = _oracle_keys(q, g, 0, "l2")
    c = (b + world - 1) // world
    for r in range(world):
        np.testing.assert_array_equal(out[r][0], full)
        assert out[r][1] == max(0, min(b, (r + 1) * c) - min(b, r * c))
