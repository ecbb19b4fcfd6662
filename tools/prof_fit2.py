"""Time the C3 fit and the C2-shape fits (n = 2000 / 10000, Gram path) once each; prints
one JSON line (for A/B runs of eigensolver variants with the diagnostic library)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "face-detection-recognization-pca_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
from eigenface import Engine  # noqa: E402

torch.cuda.set_device(0)
eng = Engine(0)
c3 = bench.fit_bench_c3(eng, False)
c2 = bench.fit_bench(eng, True)
print(json.dumps({"c3_fit_s": c3["gpu_fit_s"], "c3_iters": c3["eigensolver_iters"],
                  "c3_top3": c3["explained_variance_top3"], **{k: v for k, v in c2.items() if k != "note"}}),
      flush=True)
eng.close()
