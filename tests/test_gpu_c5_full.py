"""BASELINE.json configs[4] (C5) recognition at its own size, as a test:
1M x 512 gallery, 4096 planted 256x256 uint8 probes, the bf16 projection
(EF_MODEL_BF16) — the bench's exact workload (eigenface.synth).  Covers the wide plans at
N = 1M and KP = 512 (chunk counts, the blocked XCD deal with its serpentine k order, the
collect-pass grid) for the fp32 wide scan, the split-bf16 one (search_wide16_kernel) and
the single-bf16 screen (option 3, search_wide16_kernel<.., HI1>), L2 and cosine:

* L2: every probe finds its planted row;
* split-bf16 and bf16-screen keys == fp32-scan keys bit for bit; fused recognise == project + search;
* the exactness guarantee (tests/parity_util.py) on the GPU's (bf16-projected) features:
  every probe outside the 1e-12 tie window gets the fp64 first-arg-best row — all 4096
  against the device fp64 checker, a 256-probe subset against the CPU oracle;
* near-tie stress: a rival for every probe's best row inside fp32 / bf16 rounding, outside
  the tie window (test_gpu_c3_full.near_tie_stress), for all three scans.
"""
import numpy as np
import pytest

from test_gpu_c3_full import full_size_check, near_tie_stress

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
    return dict(mean=mean, W=W, G=G, targets=targets, P_dev=torch.from_numpy(P).cuda(), cache={})


@pytest.mark.parametrize("split", [0, 1, 3])
def test_c5_full_size(eng, c5, split):
    full_size_check(eng, c5, splits=(split,), precision="bf16")


def test_c5_near_tie_stress(eng, c5):
    near_tie_stress(eng, c5, splits=(0, 1, 3), precision="bf16")
