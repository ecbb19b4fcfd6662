"""A/B of the fit's subspace iteration (EF_OPT_FIT_CHEBYSHEV 0/1, and the fp32 coarse phase)
on bench.py's C3 fit workload (1M synthetic 128x128 faces in HBM, k = 128, StandardScaler):
time, iterations and the difference between the two results.
usage: python tools/fit_cheb_ab.py [n]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "face-detection-recognization-pca_amd"))
sys.path.insert(0, ROOT)


def main():
    import torch
    from eigenface import Engine, synth
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    side, k, r = 128, 128, 256
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
        X[a:e] = (mu + z @ B.T + 2.0 * torch.randn((e - a, d), generator=g, device=dev)).round_().clamp_(0, 255).to(torch.uint8)
    torch.cuda.synchronize()
    eng = Engine(0)
    res = {}
    modes = [(1, 1), (1, 2), (0, 1), (1, 1), (1, 2), (0, 1)]  # (chebyshev, coarse phase)
    for cheb, coarse in modes:
        eng.set_option("fit_chebyshev", cheb)
        eng.set_option("fit_fp32_coarse", coarse)
        eng.fit(X[:4096], 16, standardize=True, projection=False)
        torch.cuda.synchronize()
        t = time.perf_counter()
        r1 = eng.fit(X, k, standardize=True, projection=False)
        dt = time.perf_counter() - t
        print(f"chebyshev={cheb} coarse={coarse}: fit {dt:.4f} s, iterations {r1.iters}", flush=True)
        res[(cheb, coarse)] = r1
    a, b = res[(1, 1)], res[(0, 1)]
    ev_a, ev_b = a.eigenvalues.cpu().numpy(), b.eigenvalues.cpu().numpy()
    ca, cb = a.components.cpu().numpy(), b.components.cpu().numpy()
    s = np.sign((ca * cb).sum(1))
    print("max rel eigenvalue diff", float(np.max(np.abs(ev_a - ev_b) / ev_b)),
          "max component diff", float(np.max(np.abs(ca - cb * s[:, None]))), "sign flips", int((s < 0).sum()))
    eng.close()


if __name__ == "__main__":
    main()
