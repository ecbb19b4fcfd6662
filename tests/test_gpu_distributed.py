"""Multi-rank path with the real engine: 2 ranks share the box's one GPU (gloo for the
collective, since RCCL needs one GPU per rank); each rank holds half the gallery and
the all-reduce(MIN) of packed keys must equal the single-engine result."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import PKG, ROOT

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, G, P, mean, W, out):
    import sys
    for p in (ROOT, PKG):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from eigenface import Engine
    from eigenface.distributed import ShardedGallery, shard_range
    eng = Engine(0)
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    eng.set_model(mean, W)
    lo, hi = shard_range(len(G), rank, world)
    sg = ShardedGallery(eng, G[lo:hi], len(G), rank, world)
    Pd = torch.from_numpy(P).cuda()
    res = {}
    for metric in ("l2", "cosine"):
        res[metric] = sg.recognize_keys(Pd, metric).cpu().numpy()
    torch.cuda.synchronize()
    out[rank] = res
    eng.close()
    dist.destroy_process_group()


def test_two_ranks_one_gpu_match_single_engine():
    from eigenface import Engine, synth
    side, k, n = 32, 64, 20_000
    d = side * side
    B = synth.basis(d, k, 3)
    mean = synth.mean_face(side).astype(np.float32)
    W = B.astype(np.float32)
    G = synth.gallery_rows(0, n, k)
    G[n - 1] = G[7]  # duplicate across the shard boundary: index 7 must win
    t = np.random.default_rng(4).integers(0, n, 300)
    t[0] = 7
    P = synth.probes(t, n, k, side, B=B)
    ctx = mp.get_context("spawn")
    out = ctx.Manager().dict()
    port = _port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, G, P, mean, W, out)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
        assert p.exitcode == 0
    with Engine(0) as e:
        e.set_model(mean, W)
        e.set_gallery(G)
        for metric in ("l2", "cosine"):
            ref = e.recognize_keys(P, metric)
            for r in range(2):
                np.testing.assert_array_equal(out[r][metric], ref)
    from eigenface import decode_keys
    idx, _ = decode_keys(out[0]["l2"], "l2")
    assert idx[0] == 7
    assert (idx == t).mean() > 0.99


def _rank_sub_ulp(rank, world, port, g, q, out):
    import sys
    for p in (ROOT, PKG):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from eigenface import Engine
    from eigenface.distributed import ShardedGallery, shard_range
    eng = Engine(0)
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    lo, hi = shard_range(len(g), rank, world)
    sg = ShardedGallery(eng, g[lo:hi], len(g), rank, world)
    res = {}
    for metric, qs in (("l2", q[:2]), ("cosine", q[2:])):
        res[metric] = sg.search_keys(torch.from_numpy(qs).cuda(), metric).cpu().numpy()
    torch.cuda.synchronize()
    out[rank] = res
    eng.close()
    dist.destroy_process_group()


def test_sub_ulp_winners_across_shards_are_exact():
    """Winners in different shards whose fp64 distances (or similarities) differ by ~1e-9
    relative — the same fp32 score — must resolve by fp64 exactly as one engine over the
    whole gallery does (and as np.argmin in fp64); a MIN over fp32 keys would return the
    lower-index row."""
    from eigenface import Engine, decode_keys
    from test_distributed_cpu import sub_ulp_case
    g, q, ra, rb = sub_ulp_case()
    with Engine(0) as e:
        e.set_gallery(g)
        for metric, qs, want in (("l2", q[:2], rb[:2]), ("cosine", q[2:], rb[2:])):
            idx, _ = e.search(qs, metric)
            np.testing.assert_array_equal(idx, want)
            m = e.search_matches(qs, metric)
            np.testing.assert_array_equal(decode_keys(m["key"], metric)[0], want)
    ctx = mp.get_context("spawn")
    out = ctx.Manager().dict()
    port = _port()
    procs = [ctx.Process(target=_rank_sub_ulp, args=(r, 2, port, g, q, out)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
        assert p.exitcode == 0
    for r in range(2):
        np.testing.assert_array_equal(decode_keys(out[r]["l2"], "l2")[0], rb[:2])
        np.testing.assert_array_equal(decode_keys(out[r]["cosine"], "cosine")[0], rb[2:])


def test_match_records_carry_fp64_scores():
    """ef_search_matches / ef_recognize_matches: the record's score is the fp64 score of
    the winning row (difference-form L2 / -cosine), its key equals ef_search's."""
    from eigenface import Engine, synth
    from oracle import eigenface_oracle as orc
    side, k, n = 16, 32, 5000
    d = side * side
    B = synth.basis(d, k, 5)
    mean = synth.mean_face(side).astype(np.float32)
    G = synth.gallery_rows(0, n, k)
    t = np.random.default_rng(9).integers(0, n, 257)
    P = synth.probes(t, n, k, side, B=B)
    with Engine(0) as e:
        e.set_model(mean, B.astype(np.float32))
        e.set_gallery(G)
        for metric in ("l2", "cosine"):
            keys = e.recognize_keys(P, metric)
            m = e.recognize_matches(P, metric)
            np.testing.assert_array_equal(m["key"], keys)
            f = e.project(P)
            idx = (m["key"] & 0xFFFFFFFF).astype(np.int64)
            if metric == "l2":
                ref = ((f.astype(np.float64) - G[idx].astype(np.float64)) ** 2).sum(1)
                np.testing.assert_allclose(m["score"], ref, rtol=1e-12)
                scale = (f.astype(np.float64) ** 2).sum(1) + (G.astype(np.float64) ** 2).sum(1).max()
                np.testing.assert_allclose(m["scale"], scale, rtol=1e-5)
            else:
                ref = -orc.cosine_scores(f, G[idx]).diagonal()
                np.testing.assert_allclose(m["score"], ref, rtol=1e-12)
                assert np.all(m["scale"] == 1.0)


def test_in_library_comm_single_rank():
    """ef_comm_init with one rank (the box has one GPU; RCCL needs a GPU per rank): the
    RCCL all-gather + merge path inside ef_search / ef_recognize returns exactly the
    un-communicated result, including the sub-ulp cross-row case."""
    import torch
    torch.cuda.init()
    from eigenface import Engine
    from test_distributed_cpu import sub_ulp_case
    g, q, ra, rb = sub_ulp_case()
    with Engine(0) as ref, Engine(0) as e:
        uid = Engine.comm_unique_id()
        e.comm_init(1, 0, uid)
        assert e.comm_info() == (1, 0)
        ref.set_gallery(g)
        e.set_gallery(g)
        for metric in ("l2", "cosine"):
            np.testing.assert_array_equal(e.search_keys(q, metric), ref.search_keys(q, metric))
        e.comm_destroy()
        assert e.comm_info() == (1, 0)
