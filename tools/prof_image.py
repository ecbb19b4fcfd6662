"""Run the image-side bench sections only (ingest, template localiser, Haar detector) on
cuda:0 and print them as JSON — for rocprofv3 traces and quick A/B runs."""
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
eng.timing(True)
out = bench.image_bench(eng, False)
out["haar"] = bench.haar_bench(eng, False)
print(json.dumps(out, indent=1), flush=True)
eng.close()
