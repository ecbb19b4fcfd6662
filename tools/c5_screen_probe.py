"""C5 step with the single-bf16 screen (EF_OPT_SEARCH_SPLIT_BF16 = 3) against the split-bf16
scan (1): bench.c5_bench per option, keys checked against the fp32 side leg."""
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
dev = torch.device("cuda", 0)
eng = Engine(0)
for opt in (3, 1, 3, 1):
    r = bench.c5_bench(eng, dev, False, 10, 2, 3, 0.0, split_opt=opt)
    print(json.dumps({"opt": opt, "value": r["value"], "ms_per_step": r["ms_per_step"],
                      "scan_ms": r["roofline"]["avg_launch_ms"], "planted": r["check"]["planted_match"],
                      "keys_identical_fp32": r["scan_fp32"]["keys_identical_to_headline"]}), flush=True)
eng.close()
