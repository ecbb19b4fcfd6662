"""BASELINE.json configs[2] (C3) recognition at its own size, as a test:
1M x 128 gallery, 4096 planted 128x128 uint8 probes — the bench's exact workload
(eigenface.synth).  Covers the plan sizes, chunk counts and collect-pass grid at N = 1M
for the fp32 scan and the split-bf16 scan, L2 and cosine:

* L2: every probe finds its planted row (reference analogue: recognize_face_with_model's
  arg-best, scan-template-v4.py:270-287, on the north star's L2 metric);
* split-bf16 keys == fp32 keys bit for bit, fused recognise == project + search;
* a fixed 256-probe subset against the fp64 oracle over the whole gallery
  (oracle.l2_argmin / cosine_argmax on the GPU's fp32 features): identical rows wherever
  the fp64 runner-up is outside fp32 rounding, and the chosen row's score within it
  everywhere.
"""
import numpy as np
import pytest

from oracle import eigenface_oracle as orc

pytestmark = pytest.mark.gpu

N, SIDE, K, B = 1_000_000, 128, 128, 4096


@pytest.fixture(scope="module")
def c3():
    import torch
    from eigenface import synth
    d = SIDE * SIDE
    Bas = synth.basis(d, K, 0)
    mean = synth.mean_face(SIDE).astype(np.float32)
    W = Bas.astype(np.float32)
    G = synth.gallery_rows(0, N, K)
    targets = np.random.default_rng(2024).integers(0, N, B)
    P = synth.probes(targets, N, K, SIDE, B=Bas)
    return dict(mean=mean, W=W, G=G, targets=targets, P=P, P_dev=torch.from_numpy(P).cuda())


def _oracle_subset(f, G, metric, sub):
    """fp64 scores of the subset's probes against every gallery row, in row chunks:
    (first-best idx, best score, runner-up score), scores as 'smaller is better'."""
    f64 = f[sub].astype(np.float64)
    best = np.full(len(sub), np.inf)
    second = np.full(len(sub), np.inf)
    idx = np.zeros(len(sub), np.int64)
    if metric == "cosine":
        f64 = orc._unit_rows(f64)
    for a in range(0, len(G), 131072):
        g = G[a:a + 131072].astype(np.float64)
        if metric == "l2":
            s = (f64 ** 2).sum(1)[:, None] + (g ** 2).sum(1)[None, :] - 2.0 * (f64 @ g.T)
        else:
            s = -(f64 @ orc._unit_rows(g).T)
        part = np.partition(s, 1, axis=1)[:, :2]
        j = np.argmin(s, axis=1)  # first minimum in the chunk
        cb = s[np.arange(len(sub)), j]
        # merge the chunk's top-2 into the running top-2 (earlier chunks win exact ties)
        new_best = cb < best
        second = np.where(new_best, np.minimum(best, part[:, 1]), np.minimum(second, cb))
        idx = np.where(new_best, a + j, idx)
        best = np.where(new_best, cb, best)
    return idx, best, second


@pytest.mark.parametrize("split", [0, 1])
def test_c3_full_size(eng, c3, split):
    import torch
    from eigenface import decode_keys
    G, P_dev, targets = c3["G"], c3["P_dev"], c3["targets"]
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    try:
        eng.set_model(c3["mean"], c3["W"])
        eng.set_gallery(G)
        eng.set_option("search_split_bf16", 0)
        ref_keys = {m: eng.recognize_keys(P_dev, m).cpu().numpy() for m in ("l2", "cosine")}
        eng.set_option("search_split_bf16", split)
        f = eng.project(P_dev)
        sub = np.random.default_rng(5).choice(B, 256, replace=False)
        f_host = f.cpu().numpy()
        for metric in ("l2", "cosine"):
            keys = eng.recognize_keys(P_dev, metric).cpu().numpy()
            np.testing.assert_array_equal(keys, ref_keys[metric])  # split == fp32, fused == fused
            np.testing.assert_array_equal(eng.search_keys(f, metric).cpu().numpy(), keys)  # == project + search
            idx, score = decode_keys(keys, metric)
            if metric == "l2":
                np.testing.assert_array_equal(idx, targets)
            ref_idx, ref_best, ref_second = _oracle_subset(f_host, G, metric, sub)
            fs = f_host[sub].astype(np.float64)
            if metric == "l2":
                scale = (fs ** 2).sum(1) + (G.astype(np.float64) ** 2).sum(1).max()
                mine = ((fs - G[idx[sub]].astype(np.float64)) ** 2).sum(1)
                tol = 1e-5 * scale
            else:
                mine = -(orc._unit_rows(fs) * orc._unit_rows(G[idx[sub]])).sum(1)
                tol = np.full(len(sub), 1e-6)
            assert np.all(mine - ref_best <= tol), metric
            clear = (ref_second - ref_best) > tol
            assert clear.mean() > 0.95, (metric, clear.mean())
            np.testing.assert_array_equal(idx[sub][clear], ref_idx[clear])
    finally:
        eng.set_option("search_split_bf16", 0)
        eng.use_own_stream()
