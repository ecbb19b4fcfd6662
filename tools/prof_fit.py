"""Run the config-3 fit once (for rocprofv3 kernel traces of ef_fit)."""
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
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
out = bench.fit_bench_c3(eng, False, n=n)
print(out, flush=True)
eng.close()
