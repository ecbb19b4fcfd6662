"""Fit timing experiments (C2 Gram shapes, C3 covariance shape) under env overrides."""
import os, sys, time, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "face-detection-recognization-pca_amd"))
import numpy as np
import torch
torch.cuda.init()
from eigenface import Engine, synth
eng = Engine(0)
side, k = 128, 64
d = side * side
rng = np.random.default_rng(77)
Bm = synth.basis(d, 128, 5)
n_full = 10000
coef = rng.standard_normal((n_full, 128)) * synth.spectrum(128)
X = np.clip(np.rint(synth.mean_face(side) + coef @ Bm.T + 2.0 * rng.standard_normal((n_full, d))), 0, 255).astype(np.uint8)
Xd = torch.from_numpy(X).cuda()
ref = {}
for n in (2000, 10000):
    eng.fit(Xd[:256], 16)
    torch.cuda.synchronize()
    t = time.perf_counter(); r = eng.fit(Xd[:n], k); torch.cuda.synchronize(); dt = time.perf_counter() - t
    print(json.dumps({"env": {k_: os.environ.get(k_) for k_ in ("EF_FIT_M", "EF_FIT_PATH")}, "n": n, "s": round(dt, 4),
                      "iters": r.iters, "ev": [float(v) for v in r.eigenvalues.cpu().numpy()[[0, 31, 63]]]}), flush=True)
