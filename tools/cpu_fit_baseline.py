"""CPU leg of the C3 fit ("covariance+SVD fit sec", BASELINE.json configs[2]) to
BASELINE.md's protocol: n in {10k, 50k} faces of the C3 shape (128x128
uint8, the bench's synthetic generator: mean face + 256-component spectrum + pixel noise),
k = 128, StandardScaler + PCA (train-v4.py:126-146), median of 5 runs after 2 warm-ups,
extrapolated linearly in n to 1M ("a 1M x 16384 fp64 matrix is 131 GB").

Two CPU implementations side by side:
* ``sklearn_randomized`` — what the reference's PCA(n_components=128) ('auto') picks at
  this shape: scikit-learn's randomized solver after StandardScaler (approximate);
* ``oracle_exact_cov`` — the oracle's exact path (oracle/eigenface_oracle.py
  pca_cov_fit: fp64 covariance of the standardised data + LAPACK dsyevr for the top 128
  pairs + the training projection): the algorithm the GPU runs.  Its phases are timed
  apart: the n-dependent ones (statistics + covariance, training projection) to the full
  protocol at every n, the n-independent eigensolve of the 16384-order covariance (minutes
  per run on 16 threads) once, median of --eig-repeats after one warm-up; exact fit(n) =
  cov(n) + eigh + projection(n).

CPU only (no GPU call).  Threads: the BLAS pool as the box sets it (OPENBLAS_NUM_THREADS /
OMP_NUM_THREADS = 16 per one-GPU job); the record states the affinity set and the count.
Prints one progress line per run and the JSON at the end (also written to --out).

    python tools/cpu_fit_baseline.py --n 10000 50000 --out profiles/r05/cpu_fit_baseline.json
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "face-detection-recognization-pca_amd"))


def faces(n, side=128, r=256, seed=77):
    from eigenface import synth
    d = side * side
    B = synth.basis(d, r, 5)
    sp = synth.spectrum(r)
    mu = synth.mean_face(side)
    rng = np.random.default_rng(seed)
    X = np.empty((n, d), np.uint8)
    for a in range(0, n, 4096):
        e = min(n, a + 4096)
        pix = mu + (rng.standard_normal((e - a, r)) * sp) @ B.T + 2.0 * rng.standard_normal((e - a, d))
        X[a:e] = np.clip(np.rint(pix), 0, 255).astype(np.uint8)
    return X


def blas_threads():
    try:
        from threadpoolctl import threadpool_info
        return max(int(i.get("num_threads", 1)) for i in threadpool_info())
    except Exception:  # pragma: no cover
        return None


def run(fn, warmups, repeats, tag):
    for i in range(warmups):
        t = time.perf_counter()
        fn()
        print(f"[{tag}] warm-up {i + 1}: {time.perf_counter() - t:.2f} s", flush=True)
    ts = []
    for i in range(repeats):
        t = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t)
        print(f"[{tag}] run {i + 1}: {ts[-1]:.2f} s", flush=True)
    return ts


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs="+", default=[10_000, 50_000])
    ap.add_argument("--k", type=int, default=128)
    ap.add_argument("--warmups", type=int, default=2)
    ap.add_argument("--repeats", type=int, default=5)
    ap.add_argument("--impl", nargs="+", default=["sklearn_randomized", "oracle_exact_cov"])
    ap.add_argument("--n-full", type=int, default=1_000_000)
    ap.add_argument("--eig-repeats", type=int, default=3)
    ap.add_argument("--eigh-from", default=None, help="take the (n-independent) eigensolve timing from an earlier "
                                                     "record of this tool instead of re-measuring it")
    ap.add_argument("--merge", default=None, help="earlier record whose runs are merged into this one")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import threading

    def heartbeat():  # a single eigensolve can run for minutes: keep the log moving
        t0 = time.time()
        while True:
            time.sleep(45)
            print(f"... {time.time() - t0:.0f} s", flush=True)
    threading.Thread(target=heartbeat, daemon=True).start()
    from sklearn.decomposition import PCA
    from sklearn.preprocessing import StandardScaler
    from oracle import eigenface_oracle as orc

    res = {"what": "C3 fit CPU leg: StandardScaler + PCA k=%d on synthetic 128x128 uint8 faces "
                   "(bench.py fit_bench_c3's generator), BASELINE.md protocol" % a.k,
           "host_cpus": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0)),
           "blas_threads": blas_threads(),
           "thread_env": {v: os.environ.get(v) for v in ("OPENBLAS_NUM_THREADS", "OMP_NUM_THREADS",
                                                          "MKL_NUM_THREADS")},
           "thread_count_reason": "the GPU pool gives each one-GPU job a 16-CPU share of the host and presets "
                                  "OPENBLAS/OMP_NUM_THREADS=16 (its rules: leave them); the affinity mask spans "
                                  "the whole host, so 16 threads is the job's share, not a pinning",
           "warmups": a.warmups, "repeats": a.repeats, "runs": {}}
    if a.eigh_from:
        res["eigh"] = dict(json.load(open(a.eigh_from))["eigh"], source=a.eigh_from)
    if a.merge:
        res["runs"].update(json.load(open(a.merge))["runs"])
    for n in a.n:
        X = faces(n)
        print(f"generated {n} faces", flush=True)
        for impl in a.impl:
            if impl == "sklearn_randomized":
                def fn():
                    z = StandardScaler().fit_transform(X)
                    PCA(n_components=a.k, svd_solver="randomized", random_state=0).fit_transform(z)
            elif impl == "oracle_exact_cov":
                st = {}

                def cov():
                    st.clear()
                    st.update(orc.cov_standardised(X))
                ts_c = run(cov, a.warmups, a.repeats, f"cov n={n}")
                if "eigh" not in res:
                    c0 = st["cov"]
                    ts_e = run(lambda: orc.top_eigh(c0.copy(), a.k), 1, a.eig_repeats, "eigh d=16384")
                    res["eigh"] = {"times_s": [round(t, 3) for t in ts_e], "median_s": round(float(np.median(ts_e)), 3),
                                   "protocol": f"median of {a.eig_repeats} after 1 warm-up (n-independent)"}
                _, vt = orc.top_eigh(st["cov"], a.k)
                ts_p = run(lambda: orc.project_standardised(X, st, vt), a.warmups, a.repeats, f"proj n={n}")
                med = float(np.median(ts_c)) + res["eigh"]["median_s"] + float(np.median(ts_p))
                res["runs"][f"{impl}_n{n}"] = {"impl": impl, "n": n, "cov_times_s": [round(t, 3) for t in ts_c],
                                               "proj_times_s": [round(t, 3) for t in ts_p],
                                               "median_s": round(med, 3),
                                               "extrapolated_s_at_n_full": round(med * a.n_full / n, 1)}
                st.clear()
                continue
            else:
                raise SystemExit(f"unknown impl {impl}")
            ts = run(fn, a.warmups, a.repeats, f"{impl} n={n}")
            med = float(np.median(ts))
            res["runs"][f"{impl}_n{n}"] = {"impl": impl, "n": n, "times_s": [round(t, 3) for t in ts],
                                           "median_s": round(med, 3),
                                           "extrapolated_s_at_n_full": round(med * a.n_full / n, 1)}
        del X
    # "measured at n in {10k, 50k} and extrapolated linearly in n" — the line
    # through the two medians (the eigensolve part does not grow with n)
    for impl in a.impl:
        pts = sorted((r["n"], r["median_s"]) for r in res["runs"].values() if r["impl"] == impl)
        if len(pts) >= 2:
            (n0, t0), (n1, t1) = pts[0], pts[-1]
            slope = (t1 - t0) / (n1 - n0)
            res[f"{impl}_affine_s_at_n_full"] = round(t0 + slope * (a.n_full - n0), 1)
    print(json.dumps(res))
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
