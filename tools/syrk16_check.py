"""SYRK kernel A/B (diagnostic build, EF_SYRK16 = 0 | 5 | 6): the same fit with the 32x32x32
and the 16x16x64 int8 SYRK must give bit-identical results (the covariance is exact integer
arithmetic), then the C3 fit time per variant.  usage: EF_LIB_VARIANT=diag python tools/syrk16_check.py"""
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
    assert os.environ.get("EF_LIB_VARIANT") == "diag"
    side, k, r = 128, 128, 256
    d = side * side
    dev = torch.device("cuda", 0)
    B = torch.from_numpy(synth.basis(d, r, 5)).to(dev, torch.float32)
    sp = torch.from_numpy(synth.spectrum(r)).to(dev, torch.float32)
    mu = torch.from_numpy(synth.mean_face(side)).to(dev, torch.float32)
    n = 1_000_000
    X = torch.empty((n, d), dtype=torch.uint8, device=dev)
    g = torch.Generator(device=dev)
    g.manual_seed(77)
    for a in range(0, n, 32768):
        e = min(n, a + 32768)
        z = torch.randn((e - a, r), generator=g, device=dev) * sp
        X[a:e] = (mu + z @ B.T + 2.0 * torch.randn((e - a, d), generator=g, device=dev)).round_().clamp_(0, 255).to(torch.uint8)
    torch.cuda.synchronize()
    eng = Engine(0)
    ref = None
    for v in ["0", "5", "6"]:
        os.environ["EF_SYRK16"] = v
        small = eng.fit(X[:20000], 64, standardize=True, projection=False)
        ev = small.eigenvalues.cpu().numpy()
        comp = small.components.cpu().numpy()
        if ref is None:
            ref = (ev, comp)
        else:
            print(f"EF_SYRK16={v}: 20000 x 16384 fit identical to the 32x32x32 kernel:",
                  bool(np.array_equal(ev, ref[0]) and np.array_equal(comp, ref[1])), flush=True)
    for v in ["0", "5", "6", "0", "5", "6"]:
        os.environ["EF_SYRK16"] = v
        eng.fit(X[:4096], 16, standardize=True, projection=False)
        torch.cuda.synchronize()
        t = time.perf_counter()
        res = eng.fit(X, k, standardize=True, projection=False)
        dt = time.perf_counter() - t
        print(f"EF_SYRK16={v}: C3 fit {dt:.4f} s, iterations {res.iters}", flush=True)
    eng.close()


if __name__ == "__main__":
    main()
