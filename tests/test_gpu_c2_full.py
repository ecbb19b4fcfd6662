"""BASELINE.json configs[1] (C2) recognition at its own size, as a test:
10k x 64 gallery, 4096 planted 128x128 uint8 probes, L2 and cosine — the bench's `c2`
workload (eigenface.synth), plus the reference's own construction of the gallery: the
features of enrolled face images (train-v4.py:134 `face_features = pca.transform`), here
10k rendered faces projected by the engine.  Covers the k = 64 kernels (fp32 scan and
split-bf16 scan) at the plan sizes of a 10k-row gallery:

* L2: every probe finds its planted row;
* split-bf16 keys == fp32 keys bit for bit; fused recognise == project + search;
* the exactness guarantee (tests/parity_util.py): every probe outside the 1e-12 tie window
  gets the fp64 first-arg-best row — all 4096 against the CPU oracle's fp64 scoring;
* near-tie stress (test_gpu_c3_full.near_tie_stress) for both scans.
Reference analogue: useless/scan.py:80-130 (project, then the best-scoring gallery row).
"""
import numpy as np
import pytest

import parity_util as pu
from oracle import eigenface_oracle as orc
from test_gpu_c3_full import full_size_check, near_tie_stress

pytestmark = pytest.mark.gpu

N, SIDE, K, B = 10_000, 128, 64, 4096


@pytest.fixture(scope="module")
def c2():
    import torch
    from eigenface import synth
    d = SIDE * SIDE
    Bas = synth.basis(d, K, 0)
    mean = synth.mean_face(SIDE).astype(np.float32)
    W = Bas.astype(np.float32)
    G = synth.gallery_rows(0, N, K)
    targets = np.random.default_rng(7).integers(0, N, B)
    P = synth.probes(targets, N, K, SIDE, B=Bas)
    # enrolled images of every gallery row: the probes' rendering with other noise
    rng = np.random.default_rng(99)
    faces = np.empty((N, d), np.uint8)
    for a in range(0, N, 2000):
        pix = synth.mean_face(SIDE)[None, :] + G[a:a + 2000].astype(np.float64) @ Bas.T
        faces[a:a + 2000] = np.clip(np.rint(pix + 2.0 * rng.standard_normal(pix.shape)), 0, 255)
    return dict(mean=mean, W=W, G=G, targets=targets, P=P, P_dev=torch.from_numpy(P).cuda(), faces=faces,
                cache={})


def test_c2_full_size(eng, c2):
    full_size_check(eng, c2, splits=(0, 1))


def test_c2_near_tie_stress(eng, c2):
    near_tie_stress(eng, c2, splits=(0, 1))


def test_c2_gallery_projected_from_faces(eng, c2):
    """The gallery is the engine's projection of 10k enrolled face images (as the
    reference builds face_features); probes are other renderings of the same identities.
    Features within the projection's stated bound of the fp64 oracle; identities exact
    (planted, L2) and equal to the fp64 first-arg-best outside the tie window, both
    metrics, both scans."""
    import torch
    from eigenface import decode_keys
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    try:
        eng.set_model(c2["mean"], c2["W"])
        G = eng.project(c2["faces"])
        ref = orc.project(c2["faces"][:512], c2["mean"].astype(np.float64), c2["W"].astype(np.float64))
        bound = 2e-6 * (np.abs(c2["faces"][:512].astype(np.float64) - c2["mean"]) @ np.abs(c2["W"].astype(np.float64)))
        assert np.all(np.abs(G[:512] - ref) <= bound + 1e-6)  # test_gpu_project.py:13 bound
        eng.set_gallery(G)
        f = eng.project(c2["P_dev"]).cpu().numpy()
        gmax2 = pu.gmax2_of(G)
        for metric in ("l2", "cosine"):
            top = pu.top2(f, G, metric)
            keys0 = None
            for split in (0, 1):
                eng.set_option("search_split_bf16", split)
                keys = eng.recognize_keys(c2["P_dev"], metric).cpu().numpy()
                idx, _ = decode_keys(keys, metric)
                if metric == "l2":
                    np.testing.assert_array_equal(idx, c2["targets"])
                clear = pu.assert_exact_argbest(f, G, idx, metric, ref=top, gmax2=gmax2)
                assert clear.mean() > 0.99
                if keys0 is not None:
                    np.testing.assert_array_equal(keys, keys0)
                keys0 = keys
    finally:
        eng.set_option("search_split_bf16", 0)
        eng.use_own_stream()
