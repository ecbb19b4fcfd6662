"""BASELINE.json configs[2] (C3) recognition at its own size, as a test:
1M x 128 gallery, 4096 planted 128x128 uint8 probes — the bench's exact workload
(eigenface.synth).  Covers the plan sizes, chunk counts and collect-pass grid at N = 1M
for the fp32 scan and the split-bf16 scan, L2 and cosine:

* L2: every probe finds its planted row (reference analogue: recognize_face_with_model's
  arg-best, scan-template-v4.py:270-287, on the north star's L2 metric);
* split-bf16 keys == fp32 keys bit for bit, fused recognise == project + search;
* what the engine guarantees (tests/parity_util.py): EVERY probe whose
  fp64 top-2 gap exceeds the 1e-12 tie window gets the fp64 first-arg-best row of the whole
  gallery — all 4096 probes against an independent fp64 checker (torch fp64 GEMMs on the
  GPU), and a fixed 256-probe subset against the CPU oracle (numpy fp64);
* near-tie stress: every probe's best row gets a rival in the other half
  of the gallery whose fp64 score differs by ~1e-10..1e-7 of the scale — inside fp32
  rounding, outside the tie window — so every probe goes through the reduce -> collect ->
  fp64 resolve path; zero mismatches allowed.
"""
import numpy as np
import pytest

import parity_util as pu

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
    return dict(mean=mean, W=W, G=G, targets=targets, P=P, P_dev=torch.from_numpy(P).cuda(), cache={})


def full_size_check(eng, data, splits, precision="fp32"):
    """Shared by C3 and C5: keys equal across scans, fused == project + search, planted L2
    identities, and the exactness guarantee on all probes (device fp64 checker) and on a
    256-probe subset (CPU oracle)."""
    import torch
    from eigenface import decode_keys
    G, P_dev, targets, cache = data["G"], data["P_dev"], data["targets"], data["cache"]
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    try:
        eng.set_model(data["mean"], data["W"], precision=precision)
        eng.set_gallery(G)
        eng.set_option("search_split_bf16", 0)
        ref_keys = {m: eng.recognize_keys(P_dev, m).cpu().numpy() for m in ("l2", "cosine")}
        f_host = eng.project(P_dev).cpu().numpy()
        if "f" not in cache:
            cache["f"] = f_host
            cache["gmax2"] = pu.gmax2_of(G)
            sub = np.random.default_rng(5).choice(B, 256, replace=False)
            cache["sub"] = sub
            for m in ("l2", "cosine"):
                cache["dev", m] = pu.top2_device(f_host, G, m)
                cache["cpu", m] = pu.top2(f_host[sub], G, m)
        np.testing.assert_array_equal(f_host, cache["f"])  # the projection is deterministic
        sub, gmax2 = cache["sub"], cache["gmax2"]
        for split in splits:
            eng.set_option("search_split_bf16", split)
            f = eng.project(P_dev)
            for metric in ("l2", "cosine"):
                keys = eng.recognize_keys(P_dev, metric).cpu().numpy()
                np.testing.assert_array_equal(keys, ref_keys[metric])  # split == fp32, fused == fused
                np.testing.assert_array_equal(eng.search_keys(f, metric).cpu().numpy(), keys)  # == project + search
                idx, _ = decode_keys(keys, metric)
                if metric == "l2":
                    np.testing.assert_array_equal(idx, targets)
                pu.assert_exact_argbest(f_host, G, idx, metric, ref=cache["dev", metric], gmax2=gmax2)
                pu.assert_exact_argbest(f_host[sub], G, idx[sub], metric, ref=cache["cpu", metric], gmax2=gmax2)
    finally:
        eng.set_option("search_split_bf16", 0)
        eng.use_own_stream()


def near_tie_stress(eng, data, splits, precision="fp32"):
    """Rivals for every probe's best row (L2 and cosine), then the exactness guarantee
    on all probes under every scan, keys identical across scans."""
    import torch
    from eigenface import decode_keys
    G, P_dev, cache = data["G"], data["P_dev"], data["cache"]
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    try:
        eng.set_model(data["mean"], data["W"], precision=precision)
        eng.set_option("search_split_bf16", 0)
        f_host = eng.project(P_dev).cpu().numpy()
        eng.set_gallery(G)
        base = {m: decode_keys(eng.search_keys(f_host, m), m)[0] for m in ("l2", "cosine")}
        # anchors: the best row under each metric (they coincide for most planted probes)
        extra = np.flatnonzero(base["cosine"] != base["l2"])
        anchors = np.concatenate([base["l2"], base["cosine"][extra]])
        qs = np.concatenate([f_host, f_host[extra]])
        G2, rivals = pu.plant_rivals(G, qs, anchors, seed=11)
        gmax2 = pu.gmax2_of(G2)
        refs = {m: pu.top2_device(f_host, G2, m) for m in ("l2", "cosine")}
        for m in ("l2", "cosine"):
            ridx, best, second = refs[m]
            w = pu.window(f_host, G2, m, best, gmax2)
            gap = second - best
            # the stress is real: the best two rows are inside fp32 rounding of the scan
            # scores (L2: ~K u scale; cosine ~K u) yet outside the tie window
            fp32_res = (1e-6 * (np.abs(best) + (f_host.astype(np.float64) ** 2).sum(1) + gmax2)
                        if m == "l2" else np.full(B, 1e-6))
            tight = (gap < fp32_res) & (gap > pu.MARGIN * w)
            assert tight.mean() > 0.9, (m, tight.mean())
            # every rival or its anchor is the answer
            assert np.all(np.isin(ridx[tight], np.concatenate([anchors, rivals]))), m
        eng.set_gallery(G2)
        keys0 = None
        for split in splits:
            eng.set_option("search_split_bf16", split)
            keys = {m: eng.recognize_keys(P_dev, m).cpu().numpy() for m in ("l2", "cosine")}
            for m in ("l2", "cosine"):
                idx, _ = decode_keys(keys[m], m)
                clear = pu.assert_exact_argbest(f_host, G2, idx, m, ref=refs[m], gmax2=gmax2)
                assert clear.mean() > 0.99, (m, (~clear).sum())  # (inside the window: any row in it)
                if keys0 is not None:
                    np.testing.assert_array_equal(keys[m], keys0[m])
            keys0 = keys0 or keys
    finally:
        eng.set_option("search_split_bf16", 0)
        eng.use_own_stream()


def test_c3_full_size(eng, c3):
    full_size_check(eng, c3, splits=(0, 1))


def test_c3_near_tie_stress(eng, c3):
    near_tie_stress(eng, c3, splits=(0, 1))
