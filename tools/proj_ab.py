"""C3 fit with and without the training projection (bench.fit_bench_c3, no CPU leg):
prints the JSON line; run under rocprofv3 --kernel-trace --stats for proj_i8_kernel's time.
A/B of the projection tile: EF_LIB_VARIANT=diag EF_PROJ_TN=128|256."""
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
out = bench.fit_bench_c3(eng, False)
out.pop("cpu", None)
print(json.dumps({"tn": os.environ.get("EF_PROJ_TN", "auto"), **out}), flush=True)
eng.close()
