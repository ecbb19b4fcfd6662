"""Where a streamed JPEG ingest batch goes (bench's 4096 face crops): the host time of
each call (it returns once queued), the Python-side blob addressing, the device decode per
batch (hipEvents), and the streamed wall per batch over back-to-back calls."""
import os
import sys
import time

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "face-detection-recognization-pca_amd")]
import torch  # noqa: E402

torch.cuda.init()
import bench  # noqa: E402
from eigenface import Engine  # noqa: E402
from eigenface.engine import _pack_blobs  # noqa: E402

eng = Engine(0)
eng.timing(True)
sides = [s for grp in bench.TEMPLATE_SIDES for s in grp]
blobs = bench._face_jpegs(4096, sides)
outs = [torch.empty((4096, 4096), dtype=torch.uint8, device="cuda") for _ in range(2)]
eng.ingest_jpegs(blobs, (64, 64), "bgr", out=outs[0])
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(10):
    _pack_blobs(blobs)
print(f"_pack_blobs {1e3 * (time.perf_counter() - t0) / 10:.3f} ms", flush=True)
for reps in (1, 4, 20):
    eng.timing_reset()
    torch.cuda.synchronize()
    host = []
    t0 = time.perf_counter()
    for i in range(reps):
        a = time.perf_counter()
        eng.ingest_jpegs(blobs, (64, 64), "bgr", out=outs[i & 1])
        host.append(time.perf_counter() - a)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / reps
    ms, n = eng.timing_get("jpeg")
    rms, rn = eng.timing_get("ingest")
    print(f"reps {reps:3d}: wall {1e3 * wall:.3f} ms/batch ({4096 / wall:.0f} faces/s), host per call "
          f"min {1e3 * min(host):.3f} max {1e3 * max(host):.3f} mean {1e3 * sum(host) / reps:.3f} ms, "
          f"device decode {ms / max(n, 1):.3f} ms + resize {rms / max(rn, 1):.3f} ms per batch", flush=True)
eng.close()
