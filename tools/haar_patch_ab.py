"""Haar stage-group kernel A/B (diagnostic build): the bench's 640x480 frame through the
synthetic frontal cascade with the split form everywhere vs the LDS-patch form from stage
EF_HAAR_PATCH_FROM on (16 or 32 windows per workgroup), alternated; device ms per frame.
usage: EF_LIB_VARIANT=diag python tools/haar_patch_ab.py"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import sys, json
sys.path[:0] = [sys.argv[1], sys.argv[1] + "/face-detection-recognization-pca_amd"]
import torch
torch.cuda.init()
import bench
from eigenface import Engine
eng = Engine(0)
r = bench.haar_bench(eng, False, frames=20)
print(json.dumps({"ms_per_frame_device": r["ms_per_frame_device"], "candidates": r["candidates"]}))
'''


def run(env):
    e = dict(os.environ, **env)
    out = subprocess.run([sys.executable, "-c", CHILD, ROOT], env=e, capture_output=True, text=True, timeout=300)
    if out.returncode != 0:
        print(out.stderr[-2000:])
        raise SystemExit(out.returncode)
    return out.stdout.strip().splitlines()[-1]


assert os.environ.get("EF_LIB_VARIANT") == "diag"
cases = [("split", {}), ("patch4w32", {"EF_HAAR_PATCH_FROM": "4"}), ("patch8w32", {"EF_HAAR_PATCH_FROM": "8"}),
         ("patch14w32", {"EF_HAAR_PATCH_FROM": "14"}), ("patch8w16", {"EF_HAAR_PATCH_FROM": "8", "EF_HAAR_PATCH_WIN": "16"}),
         ("patch14w16", {"EF_HAAR_PATCH_FROM": "14", "EF_HAAR_PATCH_WIN": "16"})]
for rep in range(2):
    for name, env in cases:
        print(name, run(env), flush=True)
