"""Time a gallery scan on random (unplanted) features: 1M rows, 4096 probes.
usage: python tools/wide3_ablate.py [k] [split option]  (EF_LIB_VARIANT selects ablated
libraries: their keys are invalid, only the time is read).  Reports the scan kernel's time
and the whole search step (incl. the collect + fp64 resolve of fp32/bf16-ambiguous probes)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "face-detection-recognization-pca_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

torch.cuda.init()
from eigenface import Engine  # noqa: E402

n, b = 1_000_000, 4096
k = int(sys.argv[1]) if len(sys.argv) > 1 else 512
opt = int(sys.argv[2]) if len(sys.argv) > 2 else 1
g = torch.randn((n, k), dtype=torch.float32, device="cuda")
q = torch.randn((b, k), dtype=torch.float32, device="cuda")
eng = Engine(0)
eng.set_stream(torch.cuda.current_stream().cuda_stream)
eng.set_gallery(g)
eng.set_option("search_split_bf16", opt)
keys = torch.empty(b, dtype=torch.int64, device="cuda")
for _ in range(2):
    eng.search_keys(q, "l2", keys=keys)
torch.cuda.synchronize()
eng.timing(True)
eng.timing_reset()
t = time.perf_counter()
for _ in range(10):
    eng.search_keys(q, "l2", keys=keys)
torch.cuda.synchronize()
ms, cnt = eng.timing_get("search")
print(f"{os.environ.get('EF_LIB_VARIANT', 'base')} k={k} split={opt}: search {ms / cnt:.3f} ms/launch, wall {(time.perf_counter() - t) * 100:.3f} ms/step")
