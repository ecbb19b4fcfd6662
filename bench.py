"""Headline benchmark: faces/s recognised (projection + L2 nearest neighbour) against a
1M-row gallery, 128x128 faces, k=128 eigenfaces, probe batch 4096 (BASELINE.json
configs[2]; configs[3] when launched on N GPUs: the gallery is row-sharded across ranks,
each rank projects 1/N of the probes and one RCCL all-gather shares the features; after
the local searches one RCCL all-gather of the per-rank fp64 match records and an exact
merge pick the global match on every rank).

One step = project 4096 uint8 probe faces (p - mean).W + search the gallery + (N>1) the
two all-gathers and the merge.  Inputs are resident in HBM before timing.  Data are
synthetic (eigenface.synth): planted probes, so the step's result is also checked.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--backend nccl|gloo]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

With WORLD_SIZE unset and --gpus N > 1 the script is its own launcher: the parent process
(which makes no GPU call) starts N rank processes of this file with RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT set, waits for all of them and exits
non-zero if any rank fails.  Under torchrun, --gpus must equal WORLD_SIZE.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "face-detection-recognization-pca_amd"))

PEAK_FP32_TFLOPS = 157.3  # MI355X dense fp32 MFMA (/opt/skills/guides/MI355X_MICROARCH.md)
PEAK_BF16_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (same guide; no sparsity)

CONFIGS = {
    # name: (gallery rows, face side, k, probe batch, projection precision)
    "c3": (1_000_000, 128, 128, 4096, "fp32"),
    "c2": (10_000, 128, 64, 4096, "fp32"),
    # BASELINE.json configs[4]: 256x256 faces, k=512, bf16 projection, fp32 distances
    "c5": (1_000_000, 256, 512, 4096, "bf16"),
}


def _blas_threads():
    try:
        from threadpoolctl import threadpool_info
        info = threadpool_info()
        return max(int(i.get("num_threads", 1)) for i in info) if info else os.cpu_count()
    except Exception:  # pragma: no cover
        return os.cpu_count()


def log(*a):
    print(*a, file=sys.stderr, flush=True)


THREAD_REASON = ("BASELINE.md asks for all host cores; the GPU pool gives each one-GPU job a 16-CPU share of its "
                 "host and presets OPENBLAS/OMP/MKL_NUM_THREADS=16 (its rules: leave them, and size worker pools "
                 "to that share); the affinity mask spans the whole host (no pinning), so the job's share is "
                 "the thread count, not affinity_cpus")


def _thread_env():
    return {v: os.environ.get(v) for v in ("OPENBLAS_NUM_THREADS", "OMP_NUM_THREADS", "MKL_NUM_THREADS")}


def cpu_baseline(P, mean, W, G, targets, budget_s, warmups=2, repeats=5):
    """Oracle fp32 BLAS restatement on the host cores, bounded sample, timed to BASELINE.md's
    protocol: the same probe sample `warmups` times untimed, then the median of `repeats`
    timed runs; the BLAS thread count in use and the thread variables are recorded."""
    sys.path.insert(0, ROOT)
    from oracle import eigenface_oracle as orc
    cores = _blas_threads()
    gn = np.einsum("ij,ij->i", G, G)
    # calibrate on 32 probes, then size the sample so warm-ups + repeats fit in ~budget_s
    t = time.perf_counter()
    orc.recognize_l2_f32(P[:32], mean, W, G, gn)
    per = (time.perf_counter() - t) / 32
    b = int(min(len(P), max(32, budget_s / (warmups + repeats) / max(per, 1e-9))))
    b = max(32, (b // 32) * 32)
    for _ in range(warmups):
        orc.recognize_l2_f32(P[:b], mean, W, G, gn)
    times = []
    for _ in range(repeats):
        t = time.perf_counter()
        idx, _ = orc.recognize_l2_f32(P[:b], mean, W, G, gn)
        times.append(time.perf_counter() - t)
    dt = float(np.median(times))
    return {
        "value": b / dt,
        "unit": "faces/s",
        "cores": int(cores),
        "kind": "port",
        "sample": f"{b} probes x full {len(G)}-row gallery, fp32 NumPy/OpenBLAS "
                  f"(oracle.recognize_l2_f32), median of {repeats} runs after {warmups} warm-ups, "
                  f"{dt:.2f} s each",
        "warmups": warmups,
        "repeats": [round(b / x, 2) for x in times],
        "thread_env": _thread_env(),
        "host_cpus": os.cpu_count(),
        "affinity_cpus": len(os.sched_getaffinity(0)),
        "thread_count_reason": THREAD_REASON,
        "match": float((idx == targets[:b]).mean()),
    }


def reference_pattern(P, mean, W, G64, m, budget_s):
    """The reference's per-probe call pattern (context only): for each face
    ``scaler.transform`` + ``pca.transform`` of a (1, d) row (scan-template-v4.py:262-266)
    then ``cosine_similarity([f], face_features)`` + ``np.argmax`` (:274-275), which
    normalises a copy of the whole float64 gallery per probe (sklearn pairwise.py:1734).
    Identity StandardScaler and a PCA carrying (mean, W), so the features equal the
    benchmark's model.  Timed on up to m probes within budget_s, all host cores."""
    from sklearn.decomposition import PCA
    from sklearn.metrics.pairwise import cosine_similarity
    from sklearn.preprocessing import StandardScaler
    d, k = W.shape
    sc = StandardScaler()
    sc.mean_, sc.var_, sc.scale_ = np.zeros(d), np.ones(d), np.ones(d)
    sc.n_features_in_, sc.n_samples_seen_ = d, 2
    pca = PCA(n_components=k)
    pca.components_ = np.ascontiguousarray(W.T, dtype=np.float64)
    pca.mean_ = np.asarray(mean, dtype=np.float64)
    pca.explained_variance_ = np.ones(k)
    pca.n_components_, pca.n_features_in_, pca.n_samples_ = k, d, 2
    t = time.perf_counter()
    done = 0
    for i in range(m):
        f = pca.transform(sc.transform(P[i:i + 1].astype(np.float64)))
        int(np.argmax(cosine_similarity(f, G64)[0]))
        done += 1
        if time.perf_counter() - t > budget_s:
            break
    dt = time.perf_counter() - t
    return {"value": round(done / dt, 3), "unit": "faces/s", "cores": _blas_threads(), "kind": "port",
            "sample": f"{done} probes, one sklearn scaler/pca.transform + cosine_similarity + argmax each "
                      f"against the full {len(G64)}-row float64 gallery (scan-template-v4.py:253-287)"}


def scan_roofline(split, avg_ms, bsz, rows, k, split_opt=1):
    """Roofline of one gallery-scan launch.  fp32 scan: algorithmic 2 B N k flop against the
    fp32 MFMA peak; split-bf16 scan: its MFMA work (3 bf16 products per fp32 product, at
    the padded k) against the dense bf16 peak, plus the power-limited ceiling of a bare
    LDS-fed loop of the same MFMA shape; the bf16 screen (split_opt 3, k > 128): one bf16
    product per product, the same peak and ceiling."""
    flops_launch = 2.0 * bsz * rows * k
    kpad = next(p for p in (16, 32, 64, 128, 256, 512) if p >= k) if k <= 512 else (k + 127) // 128 * 128
    if split:
        screen = split_opt == 3 and k > 128
        mflops = (1.0 if screen else 3.0) * 2.0 * bsz * rows * kpad
        a = mflops / (avg_ms * 1e-3) / 1e12
        shape16 = split_opt != 2 and k > 64
        kname = ("search16_kernel" if shape16 else "search_kernel<S3>") if k <= 128 else \
            ("search_wide16_kernel" if shape16 else "search_wide3_kernel")
        what = (" (bf16 screen: 1 x bf16 MFMA per product, fp32 accumulation + fused arg-best, fp64-resolved)"
                if screen else " (split-bf16: 3 x bf16 MFMA per fp32 product + fused arg-best, fp64-resolved)")
        rec = {"bound": "mfma", "kernel": kname + ("<HI1>" if screen else "") + what, "achieved": round(a, 2),
               "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s", "frac": round(a / PEAK_BF16_TFLOPS, 4),
               "avg_launch_ms": round(avg_ms, 4), "mfma_flops_per_launch": mflops,
               "algorithmic_flops_per_launch": flops_launch,
               "algorithmic_TFLOPs": round(flops_launch / (avg_ms * 1e-3) / 1e12, 2)}
        ceil = bf16_ceiling("16x16x32 lds" if shape16 else "32x32x16 lds")
        if ceil:
            rec["power_limited_ceiling_TFLOPs"] = ceil[0]
            rec["frac_of_power_limited_ceiling"] = round(a / ceil[0], 4)
            rec["ceiling_source"] = ceil[1]
        return rec
    a = flops_launch / (avg_ms * 1e-3) / 1e12
    return {"bound": "mfma", "kernel": ("search_kernel" if k <= 128 else "search_wide_kernel")
            + " (fp32 MFMA distance GEMM + fused arg-best)", "achieved": round(a, 2),
            "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s", "frac": round(a / PEAK_FP32_TFLOPS, 4),
            "avg_launch_ms": round(avg_ms, 4), "flops_per_launch": flops_launch}


def c5_bench(eng, dev, with_cpu: bool, steps: int, warmup: int, repeats: int, cpu_budget: float,
             split_opt: int = 3):
    """BASELINE.json configs[4] on one GPU, as a sub-record of the default run: 1M-row
    gallery, 256x256 uint8 probes, k = 512, bf16 projection, bf16-MFMA distances with fp32
    accumulation (split_opt 3, the default: the single-bf16 screen, one bf16 MFMA per
    product; 1: the split-bf16 scan, three), identities fp64-resolved either way; the
    split-bf16 and fp32 scans on the same step as side legs whose keys must be identical;
    the bf16 projection's tolerance vs fp32; planted-match check; the CPU fp32 restatement."""
    import torch
    from eigenface import decode_keys, synth
    n, side, k, bsz, precision = CONFIGS["c5"]
    d = side * side
    t_setup = time.perf_counter()
    B = synth.basis(d, k, 0)
    mean = synth.mean_face(side).astype(np.float32)
    W = B.astype(np.float32)
    G = synth.gallery_rows(0, n, k)
    targets = np.random.default_rng(2024).integers(0, n, bsz)
    P = synth.probes(targets, n, k, side, B=B)
    stream = torch.cuda.current_stream(dev)
    eng.set_stream(stream.cuda_stream)
    eng.set_model(mean, W, precision=precision)
    eng.set_gallery(G)
    P_dev = torch.from_numpy(P).to(dev)
    opts = [split_opt] + ([1] if split_opt != 1 else []) + [0]
    keys = {o: torch.empty(bsz, dtype=torch.int64, device=dev) for o in opts}
    torch.cuda.synchronize(dev)
    setup_s = time.perf_counter() - t_setup
    legs = {}
    for opt in opts:  # headline: the bf16 scan of split_opt; side legs: split-bf16, fp32
        eng.set_option("search_split_bf16", opt)
        for _ in range(warmup):
            eng.recognize_keys(P_dev, "l2", keys=keys[opt])
        eng.timing(True)
        eng.timing_reset()
        reps = []
        for _ in range(max(1, repeats)):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for _ in range(steps):
                eng.recognize_keys(P_dev, "l2", keys=keys[opt])
            torch.cuda.synchronize(dev)
            reps.append(time.perf_counter() - t0)
        eng.timing(False)
        s_ms, s_n = eng.timing_get("search")
        p_ms, p_n = eng.timing_get("project")
        legs[opt] = (reps, s_ms / max(s_n, 1), s_n, p_ms / max(p_n, 1), p_n)
    eng.set_option("search_split_bf16", 0)
    reps, s_avg, s_n, p_avg, p_n = legs[split_opt]
    el = float(np.median(reps))
    idx, _ = decode_keys(keys[split_opt].cpu().numpy(), "l2")
    traffic, traffic_src = pmc_traffic("c5hi" if split_opt == 3 else "c5s3")
    scan_name = ("bf16 distance screen (one bf16 MFMA per product, fp32 accumulate, fp64-resolved)"
                 if split_opt == 3 else "split-bf16 distance scan (fp32 accumulate, fp64-resolved)")
    out = {"config": f"C5: gallery {n} x k={k}, {side}x{side} uint8 faces, probe batch {bsz}, metric l2, "
                     f"bf16 projection, {scan_name}",
           "value": round(bsz * steps / el, 1), "unit": "faces/s", "steps": steps, "warmup": warmup,
           "ms_per_step": round(el / steps * 1e3, 4),
           "repeats_ms_per_step": [round(r / steps * 1e3, 4) for r in reps],
           "roofline": dict(scan_roofline(True, s_avg, bsz, n, k, split_opt), traffic=traffic,
                            traffic_source=traffic_src, launches=s_n),
           "setup_s": round(setup_s, 1)}
    # the bf16 projection kernel (project_bf16_frag_kernel): 2 B d k flop per
    # launch on bf16 MFMA; algorithmic bytes = uint8 pixels + bf16 W + fp32 features
    pf = 2.0 * bsz * d * k
    ptraf, ptraf_src = pmc_traffic("c5proj")
    proj_tf = pf / (p_avg * 1e-3) / 1e12 if p_avg > 0 else None
    out["projection"] = {"kernel": "project_bf16_frag_kernel<512, 128> (W16 in MFMA-fragment order, B from L2 "
                                   "into VGPRs)", "bound": "mfma", "avg_launch_ms": round(p_avg, 4),
                         "launches": p_n, "flops_per_launch": pf,
                         "achieved": round(proj_tf, 2) if proj_tf else None, "peak": PEAK_BF16_TFLOPS,
                         "unit": "TFLOP/s", "frac": round(proj_tf / PEAK_BF16_TFLOPS, 4) if proj_tf else None,
                         "algorithmic_bytes": bsz * d + k * d * 2 + bsz * k * 4,
                         "traffic": ptraf, "traffic_source": ptraf_src}
    if split_opt != 1:
        reps1, s1_avg, s1_n, _, _ = legs[1]
        el1 = float(np.median(reps1))
        out["scan_split_bf16"] = {"value": round(bsz * steps / el1, 1), "unit": "faces/s",
                                  "ms_per_step": round(el1 / steps * 1e3, 4),
                                  "keys_identical_to_headline": bool(torch.equal(keys[1], keys[split_opt])),
                                  "roofline": dict(scan_roofline(True, s1_avg, bsz, n, k, 1), launches=s1_n)}
    reps32, s32_avg, s32_n, _, _ = legs[0]
    el32 = float(np.median(reps32))
    traffic32, src32 = pmc_traffic("c5")
    out["scan_fp32"] = {"value": round(bsz * steps / el32, 1), "unit": "faces/s",
                        "ms_per_step": round(el32 / steps * 1e3, 4),
                        "keys_identical_to_headline": bool(torch.equal(keys[0], keys[split_opt])),
                        "roofline": dict(scan_roofline(False, s32_avg, bsz, n, k), traffic=traffic32,
                                         traffic_source=src32, launches=s32_n)}
    # bf16 projection vs fp32 projection on the same step (SURVEY 8(d) C5 tolerance)
    f16 = torch.empty((bsz, k), dtype=torch.float32, device=dev)
    f32 = torch.empty_like(f16)
    k16 = eng.recognize_keys(P_dev, "l2", feats=f16).clone()
    eng.set_model(mean, W, precision="fp32")
    k32 = eng.recognize_keys(P_dev, "l2", feats=f32).clone()
    torch.cuda.synchronize(dev)
    out["bf16_projection_tolerance"] = {
        "features_max_rel_err_l2": ((f16 - f32).norm(dim=1) / f32.norm(dim=1).clamp_min(1e-30)).max().item(),
        "argmin_agreement_bf16_vs_fp32_projection": float(((k16 & 0xFFFFFFFF) == (k32 & 0xFFFFFFFF))
                                                          .float().mean().item()),
        "stated_bound": "|f_bf16 - f_fp32| <= 2^-8 sum|p - round(mu)||W| per feature (tests/test_gpu_project.py)"}
    out["check"] = {"planted_match": float((idx == targets).mean())}
    if with_cpu:
        out["cpu_baseline"] = cpu_baseline(P, mean, W, G, targets, cpu_budget)
        out["cpu_baseline"]["speedup"] = round(out["value"] / out["cpu_baseline"]["value"], 1)
    eng.use_own_stream()
    return out


def c2_bench(eng, with_cpu: bool, steps=20, repeats=5, cpu_budget=6.0):
    """BASELINE.json configs[1] recognition: 10k-row gallery, 128x128 faces, k=64, 4096
    planted probes, L2; GPU median of `repeats` x `steps` steps vs the batched fp32 CPU
    restatement and the reference's per-probe pattern."""
    import torch
    from eigenface import decode_keys, synth
    n, side, k, bsz, _ = CONFIGS["c2"]
    d = side * side
    B = synth.basis(d, k, 0)
    mean = synth.mean_face(side).astype(np.float32)
    W = B.astype(np.float32)
    G = synth.gallery_rows(0, n, k)
    targets = np.random.default_rng(7).integers(0, n, bsz)
    P = synth.probes(targets, n, k, side, B=B)
    dev = torch.device("cuda", torch.cuda.current_device())
    eng.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    eng.set_model(mean, W)
    eng.set_gallery(G)
    P_dev = torch.from_numpy(P).to(dev)
    keys = torch.empty(bsz, dtype=torch.int64, device=dev)
    for _ in range(3):
        eng.recognize_keys(P_dev, "l2", keys=keys)
    eng.timing(True)
    eng.timing_reset()
    reps = []
    for _ in range(repeats):
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        for _ in range(steps):
            eng.recognize_keys(P_dev, "l2", keys=keys)
        torch.cuda.synchronize(dev)
        reps.append(time.perf_counter() - t)
    eng.timing(False)
    s_ms, s_n = eng.timing_get("search")
    p_ms, p_n = eng.timing_get("project")
    el = float(np.median(reps))
    idx, _ = decode_keys(keys.cpu().numpy(), "l2")
    # roofline: the C2 step is projection-dominated — (p - mean).W is
    # 2 d k = 2.1 MFLOP per face, the 10k-row search 2 k N = 1.3 MFLOP per face; both fp32
    # MFMA-bound (the projection: 4096 x 16384 uint8 pixels in, 64 MB, for 8.6 GFLOP)
    p_avg, s_avg = p_ms / max(p_n, 1), s_ms / max(s_n, 1)
    pf, sf = 2.0 * bsz * d * k, 2.0 * bsz * n * k
    step_tf = (pf + sf) / (el / steps) / 1e12
    proj_tf = pf / (p_avg * 1e-3) / 1e12 if p_avg > 0 else None
    search_tf = sf / (s_avg * 1e-3) / 1e12 if s_avg > 0 else None
    out = {"config": f"C2: gallery {n} x k={k}, {side}x{side} uint8 faces, probe batch {bsz}, L2, fp32",
           "value": round(bsz * steps / el, 1), "unit": "faces/s", "ms_per_step": round(el / steps * 1e3, 4),
           "repeats_ms_per_step": [round(r / steps * 1e3, 4) for r in reps],
           "planted_match": float((idx == targets).mean()),
           "roofline": {"bound": "mfma", "kernel": "project_kernel (fp32 MFMA (p - mean).W, the step's dominant "
                                                   "kernel)",
                        "achieved": round(proj_tf, 2) if proj_tf else None, "peak": PEAK_FP32_TFLOPS,
                        "unit": "TFLOP/s", "frac": round(proj_tf / PEAK_FP32_TFLOPS, 4) if proj_tf else None,
                        "avg_launch_ms": round(p_avg, 4), "flops_per_launch": pf,
                        "search": {"kernel": "search_kernel<64>", "avg_launch_ms": round(s_avg, 4),
                                   "flops_per_launch": sf,
                                   "achieved": round(search_tf, 2) if search_tf else None,
                                   "frac": round(search_tf / PEAK_FP32_TFLOPS, 4) if search_tf else None},
                        "step_TFLOPs": round(step_tf, 2), "step_frac": round(step_tf / PEAK_FP32_TFLOPS, 4),
                        "traffic": None,
                        "note": "hipEvents on the launch stream; algorithmic flops 2 B (d k + N k) per step"}}
    if with_cpu:
        out["cpu_baseline"] = cpu_baseline(P, mean, W, G, targets, cpu_budget)
        out["cpu_baseline"]["speedup"] = round(out["value"] / out["cpu_baseline"]["value"], 1)
        out["reference_pattern"] = reference_pattern(P, mean, W, G.astype(np.float64), 256, cpu_budget)
    eng.use_own_stream()
    return out


def pmc_traffic(config):
    """HBM bytes per search launch from the newest committed rocprofv3 PMC summary of
    this config (tools/pmc_summary.py: FETCH_SIZE x2 gfx950 correction + WRITE_SIZE)."""
    import glob
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "pmc_summary*.json")), reverse=True):
        rec = json.load(open(f))
        if rec.get("config") == config:
            return rec["traffic_bytes"], os.path.relpath(f, ROOT)
    return None, None


def pmc_record(config):
    """The newest committed PMC summary whose "config" is `config` (tools/pmc_summary.py,
    tools/img_summary.py), and its path."""
    import glob
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "pmc_summary*.json")), reverse=True):
        rec = json.load(open(f))
        if rec.get("config") == config:
            return rec, os.path.relpath(f, ROOT)
    return None, None


def tmatch_executed_ops(probs, H, W, tile=128, blk=32):
    """int8 MFMA work tm_corr_kernel's tiles occupy for these maps, against the
    algorithmic 2 (H-h+1)(W-w+1) h w (DESIGN K11): per template row the band's (w + 31)
    columns rounded up to whole 32-column k-blocks, over whole output row bands — 128
    rows, and in a map's last row band with one or two live 32-row blocks 32 or 64 (the
    32 x 512 / 64 x 256 tiles of ef_image.hip tm_tile_groups) — and the map's columns
    rounded up to whole 32-column blocks (a wave runs only its live column blocks)."""
    ex = 0.0
    for _, ph, pw in probs:
        oh, ow = H - ph + 1, W - pw + 1
        kb = -(-(pw + blk - 1) // blk) * blk
        full, rem = oh // tile, oh % tile
        rows = full * tile
        if rem:
            rows += {1: 32, 2: 64}.get(-(-rem // 32), tile)
        area = rows * (-(-ow // blk) * blk)
        ex += 2.0 * area * ph * kb
    return ex


def bf16_ceiling(loop, name="bf16_clock.json"):
    """TFLOP/s a bare bf16 MFMA loop of this shape (operands re-read from LDS, 2 waves per
    SIMD, every CU busy, random data) holds under the chip's power-limited clock: the
    newest committed tools/micro/bf16_clock.cpp capture (profiles/r*/bf16_clock.json; the
    int8 loops, `bf16_clock i`, in profiles/r*/i8_clock.json)."""
    import glob
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", name)), reverse=True):
        for line in open(f):
            if line.startswith("{"):
                rec = json.loads(line)
                if rec.get("loop") == loop and rec.get("threads_per_cu") == 512:
                    return rec["tflops"], os.path.relpath(f, ROOT)
    return None


FIT_CHUNK = 32768


def c3_fit_rows(lo, hi, dev, side=128, r=256):
    """Rows [lo, hi) of the C3 fit workload (SURVEY.md §8d generator: mean face +
    256-component spectrum + N(0, 2^2) pixel noise, uint8), generated on the GPU in chunks
    of FIT_CHUNK rows, each from its own seed — any rank regenerates exactly the rows of its
    shard, so the sample-sharded fit (fit_bench_sharded) sees the single-GPU fit's data."""
    import torch
    from eigenface import synth
    d = side * side
    B = torch.from_numpy(synth.basis(d, r, 5)).to(dev, torch.float32)
    sp = torch.from_numpy(synth.spectrum(r)).to(dev, torch.float32)
    mu = torch.from_numpy(synth.mean_face(side)).to(dev, torch.float32)
    X = torch.empty((hi - lo, d), dtype=torch.uint8, device=dev)
    g = torch.Generator(device=dev)
    for c in range(lo // FIT_CHUNK, (hi + FIT_CHUNK - 1) // FIT_CHUNK):
        a, e = c * FIT_CHUNK, (c + 1) * FIT_CHUNK
        g.manual_seed(77_000 + c)
        z = torch.randn((FIT_CHUNK, r), generator=g, device=dev) * sp
        pix = mu + z @ B.T + 2.0 * torch.randn((FIT_CHUNK, d), generator=g, device=dev)
        a0, e0 = max(a, lo), min(e, hi)
        X[a0 - lo:e0 - lo] = pix[a0 - a:e0 - a].round_().clamp_(0, 255).to(torch.uint8)
        del z, pix
    torch.cuda.synchronize(dev)
    return X


def _sha(t):
    import hashlib
    a = t.cpu().numpy() if hasattr(t, "cpu") else np.asarray(t)
    return hashlib.sha1(np.ascontiguousarray(a).tobytes()).hexdigest()[:16]


def fit_bench_sharded(eng, rank, world, backend, dev, n=1_000_000, side=128, k=128, repeats=3):
    """BASELINE.json configs[3] for the fit (the fit collective): the C3
    fit workload split by samples over the ranks (rank r holds rows [n r / G, n (r + 1) / G),
    c3_fit_rows); each rank's exact integer pieces (int8 SYRK of its rows), one
    all-reduce(sum) of the pieces (RCCL int64 over xGMI; the d x d piece is 2 GiB), then the
    covariance-path fit from the sums on every rank (distributed.sharded_fit).  Timed like
    the search: barrier + synchronize around each fit, the max over ranks, median of
    `repeats` after a cold fit.  The eigenvalues' hash equals fit.c3's at N = 1 (the same
    integers give the same covariance); for n <= 100k rank 0 also runs the single-GPU fit on
    all rows and checks bit identity."""
    import torch
    import torch.distributed as dist
    from eigenface.distributed import shard_range, sharded_fit
    d = side * side
    lo, hi = shard_range(n, rank, world)
    X = c3_fit_rows(lo, hi, dev, side)

    def timed(fn):
        torch.cuda.synchronize(dev)
        dist.barrier()
        t0 = time.perf_counter()
        out = fn()
        torch.cuda.synchronize(dev)
        dist.barrier()
        el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64,
                          device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        return out, float(el.item())

    _, t_cold = timed(lambda: sharded_fit(eng, X, k, standardize=True, projection=False))
    fits = []
    for _ in range(repeats):
        res, el = timed(lambda: sharded_fit(eng, X, k, standardize=True, projection=False))
        fits.append(el)
    _, t_tr = timed(lambda: sharded_fit(eng, X, k, standardize=True, projection=True))
    out = {"config": f"C4 fit: the C3 fit workload ({n} synthetic {side}x{side} uint8 faces, k={k}, "
                     f"StandardScaler+PCA) sample-sharded over {world} ranks ({hi - lo} rows on rank {rank}), "
                     f"exact integer pieces + all-reduce(sum) ({'RCCL' if backend == 'nccl' else 'gloo'}) + "
                     "covariance-path fit on every rank",
           "gpu_fit_s": round(float(np.median(fits)), 4), "gpu_fit_s_repeats": [round(x, 4) for x in fits],
           "gpu_fit_transform_s": round(t_tr, 4), "gpu_fit_cold_s": round(t_cold, 4),
           "protocol": f"max over ranks per fit, median of {repeats} after a cold fit",
           "eigensolver_iters": res.iters,
           "explained_variance_top3": [float(v) for v in res.eigenvalues[:3].cpu().numpy()],
           "eigenvalues_sha1": _sha(res.eigenvalues), "components_sha1": _sha(res.components)}
    if n <= 100_000 and rank == 0:
        Xa = c3_fit_rows(0, n, dev, side)
        ref = eng.fit(Xa, k, standardize=True, projection=False)
        out["identical_to_single_gpu_fit"] = bool(torch.equal(ref.eigenvalues, res.eigenvalues)
                                                  and torch.equal(ref.components, res.components)
                                                  and torch.equal(ref.mean, res.mean))
        del Xa
    del X
    torch.cuda.empty_cache()
    return out


def fit_bench_c3(eng, with_cpu: bool, n=1_000_000, side=128, k=128, r=256, n_cpu=10_000, repeats=5):
    """Headline secondary metric "covariance+SVD fit sec" on config 3's shape: train-v4.py's
    train_pca_model semantics (StandardScaler + PCA, k=128) on 1M synthetic 128x128 uint8
    faces resident in HBM (generated on the GPU with torch: mean face + 256-component
    spectrum + pixel noise).  GPU: ef_fit (exact int8 covariance, fp64
    subspace eigensolve, eigenfaces) with and without the 1M x 128 training projection.
    CPU (BASELINE.md protocol): live, the solver the reference's PCA(auto)
    selects at this shape (scikit-learn randomized PCA after StandardScaler) on an n_cpu-face
    sample, median of 5 after 2 warm-ups, scaled linearly to n; beside it the committed
    tools/cpu_fit_baseline.py capture (n in {10k, 50k}, both the randomized solver and the
    oracle's exact covariance path, same protocol, same box type), which takes ~15 min and
    so is not rerun inside the bench."""
    import torch
    d = side * side
    dev = torch.device("cuda", torch.cuda.current_device())
    X = c3_fit_rows(0, n, dev, side, r)
    # first call: code paths + the context's fit workspaces (~30 GB at this shape, kept
    # for later fits, ef_trim frees them) — reported as the cold time
    t = time.perf_counter()
    eng.fit(X, k, standardize=True, projection=True)
    t_cold = time.perf_counter() - t
    # median of `repeats` fits each way (BASELINE.md protocol)
    eng.timing(True)
    eng.timing_reset()
    fits = []
    for _ in range(repeats):
        t = time.perf_counter()
        r1 = eng.fit(X, k, standardize=True, projection=False)
        fits.append(time.perf_counter() - t)
    syrk_ms, syrk_n = eng.timing_get("syrk")
    syrk_ms, syrk_n = syrk_ms / max(repeats, 1), syrk_n // max(repeats, 1)
    eng.timing(False)
    t_fit = float(np.median(fits))
    fits_tr = []
    for _ in range(repeats):
        t = time.perf_counter()
        r2 = eng.fit(X, k, standardize=True, projection=True)
        fits_tr.append(time.perf_counter() - t)
    t_fit_tr = float(np.median(fits_tr))
    ev = r1.eigenvalues.cpu().numpy()
    out = {
        "config": f"C3 fit: {n} synthetic {side}x{side} uint8 faces in HBM, k={k}, StandardScaler+PCA "
                  "(train-v4.py:126-146), exact int8 covariance + fp64 eigensolve",
        "gpu_fit_s": round(t_fit, 4),
        "gpu_fit_s_repeats": [round(x, 4) for x in fits],
        "gpu_fit_transform_s": round(t_fit_tr, 4),
        "gpu_fit_transform_s_repeats": [round(x, 4) for x in fits_tr],
        "protocol": f"median of {repeats} fits after a cold fit (code paths + the context's workspaces)",
        "gpu_fit_transform_cold_s": round(t_cold, 4),
        "eigensolver_iters": r1.iters,
        "explained_variance_top3": [float(v) for v in ev[:3]],
        "eigenvalues_sha1": _sha(r1.eigenvalues), "components_sha1": _sha(r1.components),
        "repeat_identical": bool(torch.equal(r1.components, r2.components)),
    }
    # fit roofline: the int8 SYRK (syrk_i8_kernel) is the fit's dominant kernel.  Algorithmic
    # ops = the upper triangle with its diagonal, 2 ops per multiply-add: n d (d + 1); the
    # launches' time from hipEvents on the fit's stream (EF_KERNEL_SYRK, one fit).
    if syrk_n > 0 and syrk_ms > 0:
        ops = float(n) * d * (d + 1)
        tops = ops / (syrk_ms * 1e-3) / 1e12
        roof = {"kernel": "syrk16_i8_kernel<6,4> (v_mfma_i32_16x16x64_i8, 256 x 384 tiles)", "bound": "mfma", "achieved": round(tops, 1),
                "peak": 5000.0, "unit": "TOP/s (int8)", "frac": round(tops / 5000.0, 4),
                "syrk_ms": round(syrk_ms, 3), "syrk_share_of_fit": round(syrk_ms * 1e-3 / t_fit, 3),
                "ops_per_fit": ops,
                "note": "ops = n d (d+1) (upper triangle of X'^T X', 2 per MAC); peak = 2 x the 2.5 PF bf16 "
                        "dense figure (MI355X_MICROARCH.md: I8 at 2x the BF16 rate per clock)"}
        ceil = bf16_ceiling("i8 16x16x64 lds", "i8_clock.json")
        if ceil:
            roof["power_limited_ceiling_TOPs"] = ceil[0]
            roof["frac_of_power_limited_ceiling"] = round(tops / ceil[0], 4)
            roof["ceiling_source"] = ceil[1]
        out["roofline"] = roof
    del r1, r2
    if with_cpu:
        xs = X[:n_cpu].cpu().numpy()
        del X
        torch.cuda.empty_cache()
        try:
            from sklearn.decomposition import PCA
            from sklearn.preprocessing import StandardScaler

            def cpu_fit():
                z = StandardScaler().fit_transform(xs)
                PCA(n_components=k, svd_solver="randomized", random_state=0).fit_transform(z)
            for _ in range(2):
                cpu_fit()
            ts = []
            for _ in range(5):
                t = time.perf_counter()
                cpu_fit()
                ts.append(time.perf_counter() - t)
            tc = float(np.median(ts))
            out["cpu"] = {"kind": "reference", "impl": "scikit-learn StandardScaler + PCA(randomized)",
                          "sample_faces": n_cpu, "sample_s": round(tc, 3), "repeats_s": [round(x, 3) for x in ts],
                          "protocol": "median of 5 after 2 warm-ups",
                          "extrapolated_s_at_n": round(tc * n / n_cpu, 2), "cores": _blas_threads(),
                          "host_cpus": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0)),
                          "thread_env": _thread_env(), "thread_count_reason": THREAD_REASON,
                          "note": "a different algorithm from the GPU's: the randomized solver the reference's "
                                  "PCA(auto) picks at this shape (approximate, unseeded in the reference), "
                                  "not the exact covariance + eigensolve the GPU runs; time scaled linearly "
                                  "in n from the sample"}
        except ImportError:  # pragma: no cover
            out["cpu"] = None
    out["cpu_protocol_capture"] = cpu_fit_capture()
    return out


def cpu_fit_capture():
    """The newest committed tools/cpu_fit_baseline.py record (profiles/r*/cpu_fit_baseline.json):
    the C3 fit's CPU legs at n in {10k, 50k}, sklearn randomized and the oracle's exact
    covariance path, median of 5 after 2 warm-ups, on a GPU box's host share."""
    import glob
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "cpu_fit_baseline.json")), reverse=True):
        rec = json.load(open(f))
        rec["source"] = os.path.relpath(f, ROOT)
        return rec
    return None


def fit_bench(eng, with_cpu: bool):
    """Fit on configs[1]'s shape (synthetic 10k faces 128x128, k=64; manual_pca semantics,
    Gram path) and on a 2000-face subset that the CPU oracle (NumPy/LAPACK manual_pca
    restatement) also runs."""
    from eigenface import synth
    side, k, n_full, n_sub = 128, 64, 10_000, 2000
    d = side * side
    rng = np.random.default_rng(77)
    B = synth.basis(d, 128, 5)
    coef = rng.standard_normal((n_full, 128)) * synth.spectrum(128)
    X = np.clip(np.rint(synth.mean_face(side) + coef @ B.T + 2.0 * rng.standard_normal((n_full, d))),
                0, 255).astype(np.uint8)
    out = {"config": f"C2 fit: synthetic faces {side}x{side}, k={k}, manual_pca semantics (Gram path)"}
    for n in (n_sub, n_full):
        eng.fit(X[:256], 16)  # warm the code paths
        t = time.perf_counter()
        r = eng.fit(X[:n], k)
        out[f"gpu_s_n{n}"] = round(time.perf_counter() - t, 4)
        out[f"gpu_iters_n{n}"] = r.iters
    if with_cpu:
        sys.path.insert(0, ROOT)
        from oracle import eigenface_oracle as orc
        t = time.perf_counter()
        _, _, _, lam = orc.manual_pca(X[:n_sub], k)
        out[f"cpu_s_n{n_sub}"] = round(time.perf_counter() - t, 4)
        r = eng.fit(X[:n_sub], k)
        out["eig_max_rel_err_vs_cpu"] = float(np.max(np.abs(r.eigenvalues - lam) / lam))
    out["note"] = "host X (includes the H2D copy of the uint8 faces); CPU = oracle manual_pca, all host cores"
    return out


# First five detection sizes of each lock_version model (the templates scan-template-v4.py
# loads, :45-55), from faces/lock_version/*/*_faces_detection.json: shun, ruiyi,
# Joseph_Lai, ruisheng.  Square crops.
TEMPLATE_SIDES = [[224, 232, 234, 235, 82], [217, 219, 214, 219, 224], [100] * 5, [143, 314, 130, 321, 325]]
PEAK_I8_TOPS = 5000.0   # MI355X dense int8 MFMA (2x the bf16 rate, MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0


def _face_jpegs(n, sides, seed=11):
    """n synthetic face-crop JPEGs as the reference writes them (cv2.imwrite defaults:
    baseline, quality 95, 4:2:0; detection-v4.py:64), smooth photograph-like content."""
    import io as _io
    from PIL import Image
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        s = sides[i % len(sides)]
        y, x = np.mgrid[0:s, 0:s].astype(np.float32)
        a, b, p = rng.uniform(0.03, 0.15, 3)
        img = np.stack([128 + 80 * np.sin(a * x + p + c) * np.cos(b * y - c) for c in range(3)], 2)
        img = np.clip(img + rng.normal(0, 5, img.shape), 0, 255).astype(np.uint8)
        buf = _io.BytesIO()
        Image.fromarray(img).save(buf, format="JPEG", quality=95)
        out.append(buf.getvalue())
    return out


def _host_threads():
    """The library's host worker count: the job's CPU share (OMP_NUM_THREADS, else the
    affinity mask), capped at 16 (Engine sets EF_OPT_HOST_THREADS from the same rule)."""
    from eigenface.engine import host_cpu_share
    return host_cpu_share()


def jpeg_ingest_bench(eng, with_cpu: bool, sides, n=4096, reps=20):
    """JPEG files -> grey 64x64 rows (ef_jpeg_ingest into a device tensor): a stream of
    `reps` batches, each call returning once queued, so batch i+1's host marker parse +
    destuff overlaps batch i's upload / GPU Huffman / IDCT / upsample+YCC / resize; the
    clock stops after a device synchronise.  Against per-file libjpeg-turbo decoding."""
    import torch
    blobs = _face_jpegs(n, sides)
    nbytes = sum(len(b) for b in blobs)
    dev = torch.device("cuda", torch.cuda.current_device())
    out = torch.empty((n, 4096), dtype=torch.uint8, device=dev)
    # both upload slots allocated (and the early-upload path engaged: it needs a slot already
    # sized for the batch) and the host pool's pages touched before the clock starts
    for _ in range(6):
        eng.ingest_jpegs(blobs, (64, 64), "bgr", out=out)
    torch.cuda.synchronize(dev)
    eng.timing_reset()
    t = time.perf_counter()
    for _ in range(reps):
        _, st = eng.ingest_jpegs(blobs, (64, 64), "bgr", out=out)
    torch.cuda.synchronize(dev)
    wall = (time.perf_counter() - t) / reps
    assert (st == 0).all()
    k_ms, k_n = eng.timing_get("jpeg")
    kdt = k_ms / reps * 1e-3  # device decode time per batch (the ingest decodes it in parts)
    h_ms, h_n = eng.timing_get("jpeg_host")  # host staging (parse, destuff, tables) per part
    res = {"config": f"{n} JPEG face crops {min(sides)}-{max(sides)} px (q95 4:2:0, {nbytes / n / 1024:.1f} KiB avg)"
                     " -> decode -> grey 64x64, rows on the device",
           "faces_per_s": round(n / wall, 1), "ms_per_batch": round(wall * 1e3, 3),
           "decode_ms_device": round(kdt * 1e3, 3), "decode_launches_per_batch": round(k_n / reps, 2),
           "host_parse_ms": round(h_ms / reps, 3), "host_parts_per_batch": round(h_n / reps, 2),
           "host_threads": _host_threads(), "upload_MB_per_batch": round(nbytes / 1e6, 1),
           "note": "a batch's host staging (host_parse_ms: marker parse + destuff into the pinned slot + tables, "
                   "on the job's CPU share) and its upload (the destuffed entropy words, ~the file bytes, over "
                   "PCIe, sent in 4 pieces while the batch is still being destuffed) must both finish before its "
                   "decode starts; that chain runs close to the device time (decode + resize), so the stream "
                   "runs at the larger of the two plus jitter — the gap between ms_per_batch and decode + "
                   "resize is that chain, not a device wait",
           "file_MBs": round(nbytes / wall / 1e6, 1)}
    if with_cpu:
        import io as _io
        from PIL import Image
        t = time.perf_counter()
        m = 0
        while time.perf_counter() - t < 3.0 and m < n:
            im = Image.open(_io.BytesIO(blobs[m]))
            im.load()
            m += 1
        res["cpu"] = {"faces_per_s": round(m / (time.perf_counter() - t), 1), "cores": 1, "kind": "reference",
                      "sample": f"{m} files, Pillow's libjpeg-turbo decode only (the library cv2.imread wraps)"}
    return res


def _lin_src(n_out, n_in):
    """The source pair OpenCV's INTER_LINEAR reads for each output index along one axis
    (csrc/ef_resize.hpp lin_axis: float32 offset, floor, clamp)."""
    scale = 1.0 / (n_out / n_in)
    f = ((np.arange(n_out, dtype=np.float64) + 0.5) * scale - 0.5).astype(np.float32)
    s0 = np.floor(f).astype(np.int64)
    return np.clip(s0, 0, n_in - 1), np.clip(s0 + 1, 0, n_in - 1)


def ingest_touched_bytes(offs, hs, ws, chans, oh=64, ow=64, line=128):
    """HBM bytes the fused grey + resize kernel must move for a batch: the distinct
    128-byte lines holding the source pixels INTER_LINEAR samples (2 rows x 2 columns per
    output pixel; the copy and exact-2x paths read every pixel), plus the outputs.  The
    reference's cvtColor reads every pixel; that figure is reported beside it."""
    total = 0
    for o, h, w, c in zip(offs, hs, ws, chans):
        h, w, c = int(h), int(w), int(c)
        if (h == oh and w == ow) or (h == 2 * oh and w == 2 * ow):
            rows, cols = np.arange(h), np.arange(w)
        else:
            rows = np.unique(np.concatenate(_lin_src(oh, h)))
            cols = np.unique(np.concatenate(_lin_src(ow, w)))
        first = int(o) + (rows[:, None] * w + cols[None, :]) * c
        lines = np.unique(np.concatenate([first // line, (first + c - 1) // line], axis=None))
        total += lines.size * line
    return total + len(offs) * oh * ow


def image_bench(eng, with_cpu: bool, frames=20):
    """Secondary measurements of SURVEY.md §8f ranks 2-3 on the GPU (synthetic pixels):
    ingest = 4096 BGR face crops of the reference's detection sizes (82-325 px) ->
    grey -> 64x64 (train-v4.py:59-68); tmatch = one 640x480 grey camera frame against
    4 models x 5 templates x 3 scales (scan-template-v4.py:127-200)."""
    import torch
    from eigenface.image import scaled_sizes
    rng = np.random.default_rng(3)
    sides = [s for grp in TEMPLATE_SIDES for s in grp]
    # ---- ingest
    n_img = 4096
    crops = [rng.integers(0, 256, (sides[i % len(sides)], sides[i % len(sides)], 3), dtype=np.uint8)
             for i in range(n_img)]
    src_bytes = sum(c.size for c in crops)
    dev = torch.device("cuda", torch.cuda.current_device())
    out = torch.empty((n_img, 4096), dtype=torch.uint8, device=dev)
    hs = np.array([c.shape[0] for c in crops], np.int32)
    offs = np.zeros(n_img, np.int64)
    offs[1:] = np.cumsum([c.size for c in crops])[:-1]
    dbuf = torch.from_numpy(np.concatenate([c.reshape(-1) for c in crops])).to(dev)
    chans = np.full(n_img, 3, np.int32)
    from eigenface import _native as N
    import ctypes as C

    def ingest():
        N.check(eng._h, eng._lib.ef_preprocess(eng._h, dbuf.data_ptr(), offs.ctypes.data, hs.ctypes.data,
                                               hs.ctypes.data, chans.ctypes.data, n_img, 64, 64,
                                               out.data_ptr(), N.EF_MEM_DEVICE))
    ingest()
    torch.cuda.synchronize(dev)
    eng.timing_reset()
    reps = 10
    for _ in range(reps):
        ingest()
    k_ms, k_n = eng.timing_get("ingest")
    dt = k_ms / max(k_n, 1) * 1e-3  # resize kernel, hipEvents on its stream
    # algorithmic bytes: the 128-B lines holding the sampled source pixels + 4 KiB written
    # per face (the kernel gathers 2 x 2 pixels per output); the reference's cvtColor of
    # the whole crop would read every source byte (reference_bytes)
    ib = ingest_touched_bytes(offs, hs, hs, chans)
    res = {"ingest": {
        "config": f"{n_img} BGR crops {min(sides)}-{max(sides)} px -> grey 64x64, device-resident",
        "faces_per_s": round(n_img / dt, 1), "ms_per_batch_device": round(dt * 1e3, 4),
        "algorithmic_bytes": ib, "reference_bytes": src_bytes + n_img * 4096,
        "achieved_GBs": round(ib / dt / 1e9, 1), "peak_GBs": PEAK_HBM_GBS,
        "frac": round(ib / dt / 1e9 / PEAK_HBM_GBS, 4)}}
    if with_cpu:
        sys.path.insert(0, ROOT)
        from oracle import image_oracle as io
        t = time.perf_counter()
        m = 256
        for c in crops[:m]:
            io.preprocess(c)
        res["ingest"]["cpu"] = {"faces_per_s": round(m / (time.perf_counter() - t), 1), "cores": 1,
                                "kind": "port", "sample": f"{m} crops, NumPy restatement of cvtColor+resize"}
    res["jpeg_ingest"] = jpeg_ingest_bench(eng, with_cpu, sides)
    # ---- template localiser
    H, W = 480, 640
    frame = rng.integers(0, 256, (H, W), dtype=np.uint8)
    templates, probs = [], []
    for grp in TEMPLATE_SIDES:
        for sd in grp:
            ti = len(templates)
            templates.append(rng.integers(0, 256, (sd, sd), dtype=np.uint8))
            probs += [(ti, nh, nw) for _, nw, nh in scaled_sizes(sd, sd, H, W)]
    eng.tm_prepare(templates, probs, (H, W))
    ops = sum(2.0 * (H - ph + 1) * (W - pw + 1) * ph * pw for _, ph, pw in probs)
    eng.tm_match(frame)
    eng.timing_reset()
    t = time.perf_counter()
    for _ in range(frames):
        eng.tm_match(frame)
    dt = (time.perf_counter() - t) / frames
    k_ms, k_n = eng.timing_get("tmatch")
    kdt = k_ms / max(k_n, 1) * 1e-3
    res["tmatch"] = {
        "config": f"640x480 frame, {len(templates)} templates x 3 scales = {len(probs)} TM_CCOEFF_NORMED maps",
        "frames_per_s": round(1 / dt, 2), "ms_per_frame_host": round(dt * 1e3, 4),
        "ms_per_frame_device": round(kdt * 1e3, 4),
        "algorithmic_ops": ops, "achieved_TOPS": round(ops / kdt / 1e12, 2), "peak_TOPS": PEAK_I8_TOPS,
        "frac": round(ops / kdt / 1e12 / PEAK_I8_TOPS, 4)}
    # where the gap to peak goes: executed MFMA work (tiles, band) and the counters
    ex = tmatch_executed_ops(probs, H, W)
    res["tmatch"]["executed_ops"] = ex
    res["tmatch"]["executed_to_algorithmic"] = round(ex / ops, 3)
    pm, src = pmc_record("tmatch")
    if pm:
        res["tmatch"]["tm_corr_kernel"] = {"mfma_busy_frac": round(pm["mfma_busy_frac"], 4),
                                           "clock_ghz": round(pm["clock_ghz"], 3),
                                           "avg_ms_profiled": round(pm["trace_avg_ns"] / 1e6, 4), "source": src}
    if with_cpu:
        from oracle import image_oracle as io
        from eigenface.image import scaled_sizes as ss  # noqa: F401
        t = time.perf_counter()
        ncpu = 0
        for ti, ph, pw in probs:
            if time.perf_counter() - t > 8.0:
                break
            io.match_template_fft(frame, io.resize_linear(templates[ti], (pw, ph)))
            ncpu += 1
        el = time.perf_counter() - t
        res["tmatch"]["cpu"] = {"frames_per_s": round(ncpu / len(probs) / el, 4), "cores": _blas_threads(),
                                "kind": "port", "sample": f"{ncpu}/{len(probs)} maps of one frame, "
                                "scipy FFT correlation + integral-image normalisation (OpenCV's CPU method)"}
    return res


# Stage sizes of a 25-stage frontal-face cascade like OpenCV's default one (2913 stumps);
# the cascade itself ships inside OpenCV, which is absent here, so the bench synthesises
# one of that shape and calibrates its stage thresholds so ~60 % of the windows reaching
# a stage pass it (a realistic early-rejection profile).
FRONTAL_STAGES = [9, 16, 27, 32, 52, 53, 62, 72, 83, 91, 99, 115, 127, 135, 136, 137, 159, 155, 169, 196, 197,
                  181, 199, 211, 200]


def synth_frontal_cascade(frame, n_feat=2135, seed=7, keep=0.6, n_windows=4000):
    rng = np.random.default_rng(seed)
    feats = []
    for _ in range(n_feat):
        w, h = int(rng.integers(1, 12)), int(rng.integers(1, 24))
        x, y = int(rng.integers(0, 24 - 2 * w + 1)), int(rng.integers(0, 24 - h + 1))
        feats.append([(x, y, 2 * w, h, -1.0), (x + w, y, w, h, 2.0)])
    # normalised feature values of random base-layer windows (HaarEvaluator arithmetic)
    H, W = frame.shape
    ii = np.zeros((H + 1, W + 1), np.int64)
    ii[1:, 1:] = frame.astype(np.int64).cumsum(0).cumsum(1)
    sq = np.zeros((H + 1, W + 1), np.int64)
    sq[1:, 1:] = (frame.astype(np.int64) ** 2).cumsum(0).cumsum(1)
    ys, xs = rng.integers(0, H - 24, n_windows), rng.integers(0, W - 24, n_windows)

    def box(a, x, y, w, h):
        return a[ys + y + h, xs + x + w] - a[ys + y, xs + x + w] - a[ys + y + h, xs + x] + a[ys + y, xs + x]
    area = 22.0 * 22.0
    nf = area * box(sq, 1, 1, 22, 22) - box(ii, 1, 1, 22, 22).astype(np.float64) ** 2
    vnf = (1.0 / np.sqrt(np.maximum(nf, 1.0))).astype(np.float32)
    stages, alive, fi = [], np.ones(n_windows, bool), 0
    for n in FRONTAL_STAGES:
        stumps, tot = [], np.zeros(n_windows)
        for _ in range(n):
            f = feats[fi % n_feat]
            fi += 1
            val = sum(np.float32(wt) * box(ii, x, y, w, h).astype(np.float32) for x, y, w, h, wt in f) * vnf
            thr = float(np.float32(np.median(val[alive]) if alive.any() else 0.0))
            left, right = float(np.float32(rng.uniform(-1, 0))), float(np.float32(rng.uniform(0, 1)))
            stumps.append((int((fi - 1) % n_feat), thr, left, right))
            tot += np.where(val < thr, left, right)
        sthr = float(np.float32(np.quantile(tot[alive], 1 - keep))) if alive.any() else 0.0
        alive &= tot >= sthr
        stages.append((sthr, stumps))
    return {"win": (24, 24), "features": feats, "stages": stages}


def haar_bench(eng, with_cpu: bool, frames=10):
    """detection-v4.py:50-55 on a 640x480 grey frame: detectMultiScale(1.1, 5, (30, 30))
    with a synthetic 25-stage / 2913-stump frontal-face-shaped cascade."""
    import torch  # noqa: F401
    from eigenface.haar import CascadeClassifier
    rng = np.random.default_rng(11)
    H, W = 480, 640
    yy, xx = np.mgrid[0:H, 0:W]
    f = 100 + 50 * np.sin(xx / 23.0) * np.cos(yy / 31.0) + rng.normal(0, 12, (H, W))
    frame = np.clip(np.rint(f), 0, 255).astype(np.uint8)
    casc = synth_frontal_cascade(frame)
    clf = CascadeClassifier(cascade=casc, engine=eng)
    rects, cand = clf.detect(frame, 1.1, 5, (30, 30), return_candidates=True)
    eng.timing_reset()
    t = time.perf_counter()
    for _ in range(frames):
        clf.detect(frame, 1.1, 5, (30, 30))
    dt = (time.perf_counter() - t) / frames
    k_ms, k_n = eng.timing_get("haar")
    out = {"config": "640x480 grey frame, scaleFactor 1.1, minNeighbors 5, minSize 30x30, synthetic 25-stage "
                     "2913-stump cascade (60 % pass per stage on calibration windows); the frame holds no face, so "
                     "no window survives all stages: the work is ~260k stage-0 survivors through up to 24 stages "
                     "(detections are parity-tested against the oracle in tests/test_gpu_haar.py)",
           "frames_per_s": round(1 / dt, 2), "ms_per_frame_host": round(dt * 1e3, 4),
           "ms_per_frame_device": round(k_ms / max(k_n, 1), 4), "candidates": int(len(cand)),
           "detections": int(len(rects))}
    # roofline: the stage groups are bound by the texture-address unit every integral-image
    # gather passes through (no MFMA, L2-resident tables): its busy fraction from the
    # committed PMC summary (tools/img_summary.py)
    pm, src = pmc_record("haar")
    if pm:
        out["roofline"] = {"bound": "ta", "kernel": pm["kernel"], "achieved": round(100 * pm["ta_busy_frac"], 1),
                           "peak": 100.0, "unit": "% of cycles the TA is busy", "frac": round(pm["ta_busy_frac"], 4),
                           "traffic": None, "source": src}
    if with_cpu:
        sys.path.insert(0, ROOT)
        from oracle import haar_oracle as ho
        small = frame[:120, :160]
        t = time.perf_counter()
        ho.detect_multi_scale(small, casc, 1.1, 5, (30, 30))
        out["cpu"] = {"frames_per_s_160x120": round(1 / (time.perf_counter() - t), 3), "cores": 1, "kind": "port",
                      "sample": "one 160x120 crop through the NumPy restatement (OpenCV itself is absent)"}
    return out


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(n: int, argv, timeout_s=None) -> int:
    """Start n rank processes of this script (the torchrun environment contract) from a
    parent that has made no GPU call, wait for all, and return the first non-zero exit
    code (0 when every rank succeeded).  When one rank fails the others are stopped, so
    a rank blocked in a collective cannot hang the job."""
    import subprocess
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    t0 = time.time()
    rc = 0
    alive = list(procs)
    while alive:
        for p in list(alive):
            code = p.poll()
            if code is None:
                continue
            alive.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                log(f"[launcher] rank {procs.index(p)} exited with {code}; stopping the others")
                for q in alive:
                    q.terminate()
        if timeout_s and time.time() - t0 > timeout_s and alive:
            log(f"[launcher] timeout after {timeout_s} s; stopping {len(alive)} rank(s)")
            for q in alive:
                q.terminate()
            rc = rc or 124
        time.sleep(0.05)
    for p in procs:
        p.wait()
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="torch.distributed backend for N > 1 (nccl = RCCL over xGMI; gloo exchanges through "
                         "the host and lets ranks share one GPU, for tests)")
    ap.add_argument("--launch-timeout", type=float, default=0.0,
                    help="self-launch (N > 1 without torchrun): stop every rank after this many seconds (0: none)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--repeats", type=int, default=5,
                    help="timed repeats of the K steps; value = the median repeat (BASELINE.md)")
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--metric", default="l2", choices=["l2", "cosine"])
    ap.add_argument("--cpu-budget", type=float, default=12.0, help="seconds of CPU baseline work")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-fit", action="store_true", help="skip the secondary fit timing")
    ap.add_argument("--fit-n", type=int, default=1_000_000, help="faces in the C3 / C4 fit workload")
    ap.add_argument("--fit-side", type=int, default=128, help="face side of the fit workload (tests: smaller)")
    ap.add_argument("--no-c2", action="store_true", help="skip the config-2 recognition line")
    ap.add_argument("--no-c5", action="store_true", help="skip the config-5 sub-record of the default run")
    ap.add_argument("--no-image", action="store_true", help="skip the ingest / template-localiser timing")
    ap.add_argument("--gallery", type=int, default=0, help="override the gallery size (per-rank studies)")
    ap.add_argument("--search", default=None, choices=["fp32", "split_bf16"],
                    help="headline gallery-scan arithmetic (default: fp32, the north star's; split_bf16 for "
                         "config 5, whose bf16-MFMA + fp32-accumulate arithmetic it is); the other one is timed "
                         "as a side leg")
    ap.add_argument("--no-split", action="store_true", help="skip the side leg of the other scan arithmetic")
    ap.add_argument("--split-opt", type=int, default=1, choices=[1, 2, 3],
                    help="EF_OPT_SEARCH_SPLIT_BF16 value of the split scan (2: the 32x32x16 kernel at k = 128; "
                         "3: the single-bf16 screen at k > 128)")
    ap.add_argument("--merge", default="exact", choices=["exact", "min"],
                    help="N > 1 exchange: 'exact' = all-gather of fp64 match records + exact merge (default); "
                         "'min' = one all-reduce(MIN) of packed fp32 keys (SURVEY 8e; differs only on sub-ulp "
                         "cross-shard near-ties); the other one is timed on the same step as a side record")
    ap.add_argument("--c5-opt", type=int, default=3, choices=[1, 3],
                    help="EF_OPT_SEARCH_SPLIT_BF16 value of the c5 sub-record's headline scan (3: the bf16 "
                         "screen; 1: the split-bf16 scan)")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")

    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:  # be the launcher: no torch / GPU call in this process
            sys.exit(launch_ranks(args.gpus, sys.argv[1:], args.launch_timeout or None))
        world = 1
    else:
        world = int(os.environ["WORLD_SIZE"])
        if world != args.gpus:
            ap.error(f"--gpus {args.gpus} disagrees with WORLD_SIZE={world} from the launcher")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    import torch.distributed as dist

    ndev = torch.cuda.device_count()
    if ndev < 1:
        log("bench.py: no GPU visible")
        sys.exit(2)
    if local >= ndev:
        if args.backend == "nccl":  # RCCL needs one GPU per rank
            log(f"bench.py: rank {rank} has LOCAL_RANK {local} but only {ndev} GPU(s) are visible; "
                "use --backend gloo to let ranks share a GPU")
            sys.exit(2)
        log(f"[rank {rank}] sharing GPU {local % ndev} (gloo, {ndev} GPU(s) visible)")
    dev_index = local % ndev
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    local = dev_index
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        else:
            dist.init_process_group("gloo", rank=rank, world_size=world)

    from eigenface import Engine, decode_keys, synth
    from eigenface.distributed import ShardedGallery, shard_range

    n_total, side, k, bsz, precision = CONFIGS[args.config]
    if args.gallery:
        n_total = args.gallery
    d = side * side
    lo, hi = shard_range(n_total, rank, world)

    t_setup = time.perf_counter()
    B = synth.basis(d, k, 0)
    mean = synth.mean_face(side).astype(np.float32)
    W = B.astype(np.float32)
    G = synth.gallery_rows(lo, hi, k)
    targets = np.random.default_rng(2024).integers(0, n_total, bsz)
    P = synth.probes(targets, n_total, k, side, B=B)

    eng = Engine(local)
    stream = torch.cuda.current_stream(dev)
    eng.set_stream(stream.cuda_stream)
    eng.set_model(mean, W, precision=precision)
    shard = ShardedGallery(eng, G, n_total, rank, world, merge=args.merge)
    P_dev = torch.from_numpy(P).to(dev)
    keys = torch.empty(bsz, dtype=torch.int64, device=dev)
    torch.cuda.synchronize(dev)
    log(f"[rank {rank}] setup {time.perf_counter() - t_setup:.1f}s gallery rows [{lo},{hi})")

    def step():  # project + local search + (N>1) all-gather of match records and exact merge
        shard.recognize_keys(P_dev, args.metric, keys=keys)

    def timed(step):
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize(dev)
        # R repeats of exactly K timed steps, each bracketed by barrier + synchronize; the
        # reported step time is the median repeat (max over ranks within each repeat)
        reps = []
        eng.timing(True)
        eng.timing_reset()
        for _ in range(max(1, args.repeats)):
            torch.cuda.synchronize(dev)
            if world > 1:
                dist.barrier()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                step()
            torch.cuda.synchronize(dev)
            if world > 1:
                dist.barrier()
            el = time.perf_counter() - t0
            if world > 1:
                t = torch.tensor([el], dtype=torch.float64, device=dev if args.backend == "nccl" else "cpu")
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                el = float(t.item())
            reps.append(el)
        eng.timing(False)
        return reps, eng.timing_get("search"), eng.timing_get("project")

    split_main = (args.search or ("split_bf16" if args.config == "c5" else "fp32")) == "split_bf16"
    split_val = args.split_opt
    eng.set_option("search_split_bf16", split_val if split_main else 0)
    reps, (s_ms, s_n), (p_ms, p_n) = timed(step)
    el = float(np.median(reps))

    idx, best = decode_keys(keys.cpu().numpy(), args.metric)
    match = float((idx == targets).mean())
    exchange_ms = None
    if world > 1:  # the step's collectives alone (upper bound of their share; max over ranks)
        t = torch.tensor([shard.exchange_ms(bsz, k, dev)], dtype=torch.float64,
                         device=dev if args.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        exchange_ms = float(t.item())
    other_merge = None
    if world > 1:  # the other exchange on the same step: exact record merge <-> one all-reduce(MIN)
        main_keys = keys.clone()
        shard.merge = "min" if args.merge == "exact" else "exact"
        reps_o, _, _ = timed(step)
        xo = torch.tensor([shard.exchange_ms(bsz, k, dev)], dtype=torch.float64,
                          device=dev if args.backend == "nccl" else "cpu")
        dist.all_reduce(xo, op=dist.ReduceOp.MAX)
        other_merge = {"merge": shard.merge, "ms_per_step": round(float(np.median(reps_o)) / args.steps * 1e3, 4),
                       "exchange_ms_per_step": round(float(xo.item()), 4),
                       "keys_identical": bool(torch.equal(keys, main_keys))}
        shard.merge = args.merge
        keys.copy_(main_keys)
    ranks_agree = None
    if world > 1:  # every rank must hold the same merged keys
        h = torch.tensor([int(np.bitwise_xor.reduce(keys.cpu().numpy() * np.int64(0x9E3779B1)))
                          & 0x7FFFFFFFFFFFFFFF], dtype=torch.int64,
                         device=dev if args.backend == "nccl" else "cpu")
        lo_t, hi_t = h.clone(), h.clone()
        dist.all_reduce(lo_t, op=dist.ReduceOp.MIN)
        dist.all_reduce(hi_t, op=dist.ReduceOp.MAX)
        ranks_agree = bool(lo_t.item() == hi_t.item())

    host_rate = host_same = None
    if world == 1:  # PCIe-inclusive rate (never `value`)
        eng.use_own_stream()
        eng.recognize_keys(P, args.metric)
        t = time.perf_counter()
        for _ in range(3):
            hk = eng.recognize_keys(P, args.metric)
        host_rate = 3 * bsz / (time.perf_counter() - t)
        host_same = bool(np.array_equal(hk, keys.cpu().numpy()))

    split_leg = None
    if world == 1 and not args.no_split:
        # the other scan precision on the same step: split-bf16 when the headline is fp32
        # (and vice versa); its keys must equal the headline's bit for bit
        eng.set_stream(stream.cuda_stream)
        eng.set_option("search_split_bf16", 0 if split_main else split_val)
        keys2 = torch.empty_like(keys)

        def step2():
            shard.recognize_keys(P_dev, args.metric, keys=keys2)

        reps2, (s2_ms, s2_n), _ = timed(step2)
        eng.set_option("search_split_bf16", split_val if split_main else 0)
        split_leg = {"scan": "split_bf16" if not split_main else "fp32", "reps": reps2,
                     "search_avg_ms": s2_ms / max(s2_n, 1), "launches": s2_n,
                     "keys_identical": bool(torch.equal(keys2, keys))}

    fit_sharded = None
    if world > 1 and not args.no_fit:  # every rank: the sample-sharded fit is collective
        eng.set_stream(stream.cuda_stream)
        fit_sharded = fit_bench_sharded(eng, rank, world, args.backend, dev, n=args.fit_n, side=args.fit_side)

    tol = None
    if world == 1 and precision == "bf16":
        # the bf16 projection's tolerance vs fp32 — max relative feature
        # error and the argmin agreement rate of the two projections on the same step
        eng.set_stream(stream.cuda_stream)
        f16 = torch.empty((bsz, k), dtype=torch.float32, device=dev)
        f32 = torch.empty_like(f16)
        k16 = eng.recognize_keys(P_dev, args.metric, feats=f16).clone()
        eng.set_model(mean, W, precision="fp32")
        k32 = eng.recognize_keys(P_dev, args.metric, feats=f32).clone()
        eng.set_model(mean, W, precision=precision)
        torch.cuda.synchronize(dev)
        rel = ((f16 - f32).norm(dim=1) / f32.norm(dim=1).clamp_min(1e-30)).max().item()
        tol = {"features_max_rel_err_l2": rel,
               "features_max_abs_err_over_max_abs": ((f16 - f32).abs().max() / f32.abs().max()).item(),
               "argmin_agreement_bf16_vs_fp32_projection": float(((k16 & 0xFFFFFFFF) == (k32 & 0xFFFFFFFF))
                                                                 .float().mean().item()),
               "stated_bound": "|f_bf16 - f_fp32| <= 2^-8 sum|p - round(mu)||W| per feature (tests/test_gpu_project.py)"}

    if rank == 0:
        ms_step = el / args.steps * 1e3
        value = bsz * args.steps / el
        search_avg_ms = s_ms / max(s_n, 1)

        def roof(split, avg_ms):
            return scan_roofline(split, avg_ms, bsz, hi - lo, k, args.split_opt)

        def traffic_key(split):  # the committed PMC summary of this scan (pmc_summary.py configs)
            if not split:
                return args.config
            return args.config + ("hi" if args.split_opt == 3 and k > 128 else "s3")

        traffic, traffic_src = pmc_traffic(traffic_key(split_main)) if world == 1 else (None, None)
        rec = {
            "metric": "faces/sec recognized (projection+NN) @1M-gallery k=128" if args.config == "c3"
                      else f"faces/sec recognized (projection+NN) @{n_total}-gallery k={k}",
            "value": round(value, 1),
            "unit": "faces/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 4),
            "repeats_ms_per_step": [round(r / args.steps * 1e3, 4) for r in reps],
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": ("f32" if precision == "fp32" else "bf16 projection, f32 distance")
                     if not split_main else f"{precision} projection, split-bf16 (hi+lo) distance scan, f64 resolve",
            "data": "synthetic (eigenface.synth planted probes; gallery = eigen-coefficients)",
            "config": {
                "workload": f"{args.config.upper()}: gallery {n_total} x k={k}, {side}x{side} uint8 faces, "
                            f"probe batch {bsz}, metric {args.metric}, projection {precision}",
                "gallery": n_total, "face": f"{side}x{side}", "k": k, "batch": bsz,
                "parallelism": (f"gallery row-shard x{world}: projection split + "
                                f"{'RCCL' if args.backend == 'nccl' else 'gloo (host)'} all-gather of features, "
                                "local search, all-gather of fp64 match records + exact merge")
                               if world > 1 else "1 GPU",
                "rows_per_rank": hi - lo,
                "backend": args.backend if world > 1 else None,
            },
            "roofline": dict(roof(split_main, search_avg_ms), traffic=traffic, traffic_source=traffic_src,
                             launches=s_n),
            "project_avg_ms": round(p_ms / max(p_n, 1), 4),
            "exchange_ms_per_step": round(exchange_ms, 4) if exchange_ms is not None else None,
            "exchange_share_of_step": round(exchange_ms / ms_step, 4) if exchange_ms is not None else None,
            "merge": args.merge if world > 1 else None,
            "other_merge": other_merge,
            "host_buffer_faces_per_s": round(host_rate, 1) if host_rate else None,
            "check": {"planted_match": match, "ranks_agree": ranks_agree, "host_buffer_keys_identical": host_same},
        }
        if tol:
            rec["bf16_projection_tolerance"] = tol
        if split_leg:
            el2 = float(np.median(split_leg["reps"]))
            rec["scan_" + split_leg["scan"]] = {
                "value": round(bsz * args.steps / el2, 1), "unit": "faces/s",
                "ms_per_step": round(el2 / args.steps * 1e3, 4),
                "repeats_ms_per_step": [round(r / args.steps * 1e3, 4) for r in split_leg["reps"]],
                "keys_identical_to_headline": split_leg["keys_identical"],
                "roofline": dict(roof(split_leg["scan"] == "split_bf16", split_leg["search_avg_ms"]),
                                 launches=split_leg["launches"],
                                 **dict(zip(("traffic", "traffic_source"),
                                            pmc_traffic(traffic_key(not split_main))))),
            }
        if world == 1 and not args.no_cpu:
            rec["cpu_baseline"] = cpu_baseline(P, mean, W, G, targets, args.cpu_budget)
            rec["cpu_baseline"]["reference_pattern"] = reference_pattern(P, mean, W, G.astype(np.float64), 16,
                                                                         args.cpu_budget)
        else:
            rec["cpu_baseline"] = None
        if world == 1 and args.config == "c3" and not args.no_c2:
            rec["c2"] = c2_bench(eng, not args.no_cpu)
        if world == 1 and args.config == "c3" and not args.no_c5:
            rec["c5"] = c5_bench(eng, dev, not args.no_cpu, args.steps, args.warmup, args.repeats,
                                 min(args.cpu_budget, 8.0), args.c5_opt)
        if world == 1 and not args.no_fit:
            rec["fit"] = {"c3": fit_bench_c3(eng, not args.no_cpu, n=args.fit_n, side=args.fit_side),
                          "c2": fit_bench(eng, not args.no_cpu)}
        if fit_sharded is not None:
            rec["fit"] = {"c4": fit_sharded}
        if world == 1 and not args.no_image:
            eng.use_own_stream()
            eng.timing(True)
            rec.update(image_bench(eng, not args.no_cpu))
            rec["haar"] = haar_bench(eng, not args.no_cpu)
            eng.timing(False)
        for key in ("fit", "c5"):  # the largest sub-records last: a tail of stdout shows them whole
            if key in rec:
                rec[key] = rec.pop(key)
        print(json.dumps(rec), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
