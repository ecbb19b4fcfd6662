"""The sample-sharded fit (the fit collective; include/eigenface.h
ef_fit_shard_stats / ef_fit_from_stats / ef_fit_transform): the exact integer pieces of
every shard, summed, give the covariance of the whole set, so the fit from the sums must
equal Engine.fit on the concatenated rows BIT FOR BIT (mean, var, scale, components,
eigenvalues, total variance) and the per-shard training projections must equal its
projection rows.  Shards are uneven and include an empty one; host and device forms; the
1M-face C3 workload in 4 shards; and bench.py's N > 1 sharded fit (2 ranks sharing the
GPU over gloo)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT
from oracle import eigenface_oracle as orc

pytestmark = pytest.mark.gpu


def _assert_same(a, b):
    for f in ("mean", "var", "scale", "components", "eigenvalues"):
        x, y = getattr(a, f), getattr(b, f)
        x = x.cpu().numpy() if hasattr(x, "cpu") else np.asarray(x)
        y = y.cpu().numpy() if hasattr(y, "cpu") else np.asarray(y)
        assert np.array_equal(x, y), f
    assert a.total_var == b.total_var and a.k == b.k and a.iters == b.iters


@pytest.mark.parametrize("standardize", [False, True])
def test_sharded_pieces_equal_the_whole_fit_host(eng, standardize):
    x, _ = orc.synth_faces(3001, 32, r=40, seed=19)   # n = 3001 >= d = 1024: covariance path
    ref = eng.fit(x, 24, standardize=standardize, projection=True)
    cuts = [0, 700, 700, 1999, 3001]                  # uneven, one empty shard
    pieces = [eng.fit_shard_stats(x[a:b]) for a, b in zip(cuts[:-1], cuts[1:])]
    s1, s2, cr = (sum(p[i] for p in pieces) for i in range(3))
    res = eng.fit_from_stats(s1, s2, cr, len(x), 24, standardize=standardize)
    _assert_same(res, ref)
    proj = np.concatenate([eng.fit_transform_rows(x[a:b], res, standardize) for a, b in zip(cuts[:-1], cuts[1:])
                           if b > a])
    assert np.array_equal(proj, ref.projection)
    # and the oracle's exact-covariance fit on the same rows (train-v4.py semantics)
    if standardize:
        o = orc.pca_cov_fit(x, 24, standardize=True)
        np.testing.assert_allclose(res.eigenvalues, o["explained_variance_"], rtol=1e-9)
        np.testing.assert_allclose(res.components, o["components_"], atol=1e-7)


def test_sharded_pieces_device_and_guards(eng):
    import torch
    x, _ = orc.synth_faces(2000, 32, r=40, seed=23)
    xd = torch.from_numpy(x).cuda()
    ref = eng.fit(xd, 16, standardize=True, projection=True)
    p0, p1 = eng.fit_shard_stats(xd[:1234]), eng.fit_shard_stats(xd[1234:])
    s1, s2, cr = (p0[i] + p1[i] for i in range(3))
    res = eng.fit_from_stats(s1, s2, cr, 2000, 16, standardize=True)
    _assert_same(res, ref)
    proj = torch.cat([eng.fit_transform_rows(xd[:1234], res, True), eng.fit_transform_rows(xd[1234:], res, True)])
    assert torch.equal(proj, ref.projection)
    # the Gram path (n_total < d) is not shardable by samples: refused before any GPU work
    from eigenface import EigenfaceError
    with pytest.raises(EigenfaceError):
        eng.fit_from_stats(s1, s2, cr, 999, 16)


def test_sharded_fit_c3_size_in_four_shards(eng):
    """The 1M-face C3 fit workload (bench.py c3_fit_rows) in four shards of 250k: the fit
    from the summed pieces is bit-identical to the single fit."""
    import torch
    sys.path.insert(0, ROOT)
    import bench
    dev = torch.device("cuda", 0)
    X = bench.c3_fit_rows(0, 1_000_000, dev)
    ref = eng.fit(X, 128, standardize=True, projection=False)
    tot = None
    for a in range(0, 1_000_000, 250_000):
        p = eng.fit_shard_stats(X[a:a + 250_000])
        tot = list(p) if tot is None else [t + q for t, q in zip(tot, p)]
        del p
    res = eng.fit_from_stats(*tot, 1_000_000, 128, standardize=True)
    _assert_same(res, ref)
    del X, tot
    torch.cuda.empty_cache()


def test_bench_sharded_fit_two_ranks_one_gpu():
    """bench.py at N = 2 (gloo, both ranks on this GPU) runs the sample-sharded fit
    (fit_bench_sharded) and rank 0 checks it bit for bit against the single-GPU fit."""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo",
                        "--gallery", "100000", "--no-cpu", "--no-image", "--no-c2", "--no-split", "--steps", "2",
                        "--warmup", "1", "--repeats", "1", "--fit-n", "30000", "--fit-side", "64",
                        "--launch-timeout", "240"], capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    rec = json.loads(lines[-1])
    f = rec["fit"]["c4"]
    assert f["identical_to_single_gpu_fit"] is True
    assert f["gpu_fit_s"] > 0 and len(f["gpu_fit_s_repeats"]) == 3
