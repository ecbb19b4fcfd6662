"""BASELINE.json configs[4] (C5) recognition at its own size, as a test:
1M x 512 gallery, 4096 planted 256x256 uint8 probes, the bf16 projection
(EF_MODEL_BF16) — the bench's exact workload (eigenface.synth).  Covers the wide plans at
N = 1M and KP = 512 (chunk counts, the blocked XCD deal with its serpentine k order, the
collect-pass grid) for the fp32 wide scan, the split-bf16 one (search_wide16_kernel) and
the single-bf16 screen (option 3, search_wide16_kernel<.., HI1>), L2 and cosine:

* L2: every probe finds its planted row;
* split-bf16 and bf16-screen keys == fp32-scan keys bit for bit; fused recognise == project + search;
* a fixed 256-probe subset against the fp64 oracle over the whole gallery on the GPU's
  (bf16-projected) features: identical rows wherever the fp64 runner-up is outside fp32
  rounding, and the chosen row's score within it everywhere.
"""
import numpy as np
import pytest

from oracle import eigenface_oracle as orc
from test_gpu_c3_full import _oracle_subset

pytestmark = pytest.mark.gpu

N, SIDE, K, B = 1_000_000, 256, 512, 4096


@pytest.fixture(scope="module")
def c5():
    import torch
    from eigenface import synth
    d = SIDE * SIDE
    Bas = synth.basis(d, K, 0)
    mean = synth.mean_face(SIDE).astype(np.float32)
    W = Bas.astype(np.float32)
    G = synth.gallery_rows(0, N, K)
    targets = np.random.default_rng(2024).integers(0, N, B)
    P = synth.probes(targets, N, K, SIDE, B=Bas)
    return dict(mean=mean, W=W, G=G, targets=targets, P_dev=torch.from_numpy(P).cuda())


@pytest.mark.parametrize("split", [0, 1, 3])
def test_c5_full_size(eng, c5, split):
    import torch
    from eigenface import decode_keys
    G, P_dev, targets = c5["G"], c5["P_dev"], c5["targets"]
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    try:
        eng.set_model(c5["mean"], c5["W"], precision="bf16")
        eng.set_gallery(G)
        eng.set_option("search_split_bf16", 0)
        ref_keys = {m: eng.recognize_keys(P_dev, m).cpu().numpy() for m in ("l2", "cosine")}
        eng.set_option("search_split_bf16", split)
        f = eng.project(P_dev)
        sub = np.random.default_rng(5).choice(B, 256, replace=False)
        f_host = f.cpu().numpy()
        for metric in ("l2", "cosine"):
            keys = eng.recognize_keys(P_dev, metric).cpu().numpy()
            np.testing.assert_array_equal(keys, ref_keys[metric])  # split == fp32
            np.testing.assert_array_equal(eng.search_keys(f, metric).cpu().numpy(), keys)  # == project + search
            idx, _ = decode_keys(keys, metric)
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
