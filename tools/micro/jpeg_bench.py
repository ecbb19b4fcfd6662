"""JPEG ingest timing alone (bench.py's jpeg_ingest section) for decoder iterations."""
import json
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "face-detection-recognization-pca_amd")]
import torch  # noqa: E402

torch.cuda.init()
import bench  # noqa: E402
from eigenface import Engine  # noqa: E402

eng = Engine(0)
eng.timing(True)
sides = [s for grp in bench.TEMPLATE_SIDES for s in grp]
print(json.dumps(bench.jpeg_ingest_bench(eng, "--cpu" in sys.argv, sides)), flush=True)
