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
