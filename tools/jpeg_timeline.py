"""The streamed JPEG ingest under a kernel + memory-copy trace: 6 warm-up calls, then 20
back-to-back calls of bench's 4096 face crops (timing hooks off), so the trace shows where
the device idles between batches.  Run under rocprofv3 (tools/r06_jpeg_timeline.sh)."""
import gc
import os
import sys
import time

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "face-detection-recognization-pca_amd")]
import torch  # noqa: E402

torch.cuda.init()
import bench  # noqa: E402
from eigenface import Engine  # noqa: E402

eng = Engine(0)
if os.environ.get("JT_THREADS"):
    eng.set_option("host_threads", int(os.environ["JT_THREADS"]))
sides = [s for grp in bench.TEMPLATE_SIDES for s in grp]
blobs = bench._face_jpegs(4096, sides)
out = torch.empty((4096, 4096), dtype=torch.uint8, device="cuda")
for _ in range(6):
    eng.ingest_jpegs(blobs, (64, 64), "bgr", out=out)
torch.cuda.synchronize()
if os.environ.get("JT_NOGC"):
    gc.disable()
t0 = time.perf_counter()
host = []
for _ in range(int(os.environ.get('JT_REPS', 20))):
    a = time.perf_counter()
    eng.ingest_jpegs(blobs, (64, 64), "bgr", out=out)
    host.append(1e3 * (time.perf_counter() - a))
torch.cuda.synchronize()
print(f"wall {1e3 * (time.perf_counter() - t0) / len(host):.3f} ms/batch", flush=True)
print("host ms per call:", " ".join(f"{h:.2f}" for h in host), flush=True)
eng.close()
