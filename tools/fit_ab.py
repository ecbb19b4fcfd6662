"""C3 fit A/B between library builds (EF_LIB_VARIANT selects libeigenface_<tag>.so; unset =
the product library): bench.py's C3 fit workload (1M synthetic 128x128 faces in HBM,
k = 128, StandardScaler), one cold fit then the median of `reps` timed fits, the
eigensolver iteration count, and the result saved for a bit-for-bit comparison.
usage: python tools/fit_ab.py <out.npz> [reps]        (prints one JSON line)"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "face-detection-recognization-pca_amd"))


def main():
    import torch
    from eigenface import Engine, synth
    out = sys.argv[1]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    n, side, k, r = 1_000_000, 128, 128, 256
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
        X[a:e] = (mu + z @ B.T + 2.0 * torch.randn((e - a, d), generator=g, device=dev)).round_().clamp_(0, 255) \
            .to(torch.uint8)
    del B, z
    torch.cuda.synchronize()
    eng = Engine(0)
    eng.fit(X, k, standardize=True, projection=False)  # cold: code paths + workspaces
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t = time.perf_counter()
        res = eng.fit(X, k, standardize=True, projection=False)
        ts.append(time.perf_counter() - t)
    np.savez(out, eigenvalues=res.eigenvalues.cpu().numpy(), components=res.components.cpu().numpy())
    print(json.dumps({"variant": os.environ.get("EF_LIB_VARIANT", "product"), "median_s": float(np.median(ts)),
                      "fits_s": [round(x, 4) for x in ts], "iters": res.iters}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
