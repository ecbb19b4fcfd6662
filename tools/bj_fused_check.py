"""A/B of a fit-path diagnostic switch whose two settings must give bit-identical fits
(diagnostic build): EF_BJ_FUSED (block-Jacobi rounds as one launch: the solve recomputing
its off-diagonal blocks, the previous round's apply alongside, vs two launches),
EF_FINALIZE4 (the 4-column covariance finalize vs one column per thread).  Four fit
shapes must agree bit for bit; then the C3 fit time of both settings, alternated.
usage: EF_LIB_VARIANT=diag python tools/bj_fused_check.py [VAR]   (default EF_BJ_FUSED)"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "face-detection-recognization-pca_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from eigenface import Engine, synth  # noqa: E402

torch.cuda.set_device(0)
eng = Engine(0)
rng = np.random.default_rng(3)
VAR = sys.argv[1] if len(sys.argv) > 1 else "EF_BJ_FUSED"


def fit(X, k, std, fused):
    os.environ[VAR] = str(fused)
    r = eng.fit(X, k, standardize=std, projection=False)
    return np.asarray(r.components), np.asarray(r.eigenvalues), r.iters


ok = True
for (n, d, k, std) in [(3000, 640, 200, False), (900, 4096, 300, True), (30000, 4096, 128, True),
                       (20000, 16384, 128, True)]:
    basis = rng.standard_normal((64, d)) * np.linspace(40, 1, 64)[:, None]
    X = np.clip(128 + rng.standard_normal((n, 64)) @ basis / 8 + rng.standard_normal((n, d)) * 3, 0, 255)
    X = X.astype(np.uint8)
    c0, e0, i0 = fit(X, k, std, 0)
    c1, e1, i1 = fit(X, k, std, 1)
    same = np.array_equal(c0, c1) and np.array_equal(e0, e1) and i0 == i1
    ok &= same
    print(f"n={n} d={d} k={k} std={std}: identical={same} iters {i0}/{i1} "
          f"max|dc|={np.abs(c0 - c1).max():.3e} max|de|/e0={np.abs(e0 - e1).max() / e0[0]:.3e}", flush=True)

# C3 fit time (1M x 128x128, k = 128), alternated
side, n, r = 128, 1_000_000, 256
d = side * side
dev = torch.device("cuda", 0)
B = torch.from_numpy(synth.basis(d, r, 5)).to(dev, torch.float32)
sp = torch.from_numpy(synth.spectrum(r)).to(dev, torch.float32)
mu = torch.from_numpy(synth.mean_face(side)).to(dev, torch.float32)
X = torch.empty((n, d), dtype=torch.uint8, device=dev)
g = torch.Generator(device=dev)
g.manual_seed(77)
for a in range(0, n, 32768):
    e = min(n, a + 32768)
    z = torch.randn((e - a, r), generator=g, device=dev) * sp
    pix = mu + z @ B.T + 2.0 * torch.randn((e - a, d), generator=g, device=dev)
    X[a:e] = pix.round_().clamp_(0, 255).to(torch.uint8)
    del z, pix
torch.cuda.synchronize()
eng.fit(X, 128, standardize=True, projection=False)  # workspaces
res = {0: [], 1: []}
comp = {}
for rep in range(3):
    for fused in (1, 0):
        os.environ[VAR] = str(fused)
        torch.cuda.synchronize()
        t = time.perf_counter()
        rr = eng.fit(X, 128, standardize=True, projection=False)
        res[fused].append(time.perf_counter() - t)
        comp[fused] = rr.components.cpu().numpy() if hasattr(rr.components, "cpu") else np.asarray(rr.components)
same = np.array_equal(comp[0], comp[1])
ok &= same
print(f"C3 fit s: {VAR}=1 {[round(x, 4) for x in res[1]]} {VAR}=0 {[round(x, 4) for x in res[0]]} "
      f"median {np.median(res[1]):.4f} vs {np.median(res[0]):.4f}; identical={same}", flush=True)
eng.close()
print("ALL_IDENTICAL" if ok else "MISMATCH", flush=True)
