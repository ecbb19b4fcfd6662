"""Host/device breakdown of the JPEG ingest path on the bench's 4096 face crops, over
entropy-chunk sizes (EF_OPT_JPEG_CHUNK_BITS; 0 = auto)."""
import os
import sys
import time

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "face-detection-recognization-pca_amd")]
import torch  # noqa: E402

torch.cuda.init()
import bench  # noqa: E402
from eigenface import Engine  # noqa: E402
from eigenface.engine import _pack_blobs, jpeg_info  # noqa: E402

eng = Engine(0)
eng.timing(True)
sides = [s for grp in bench.TEMPLATE_SIDES for s in grp]
blobs = bench._face_jpegs(4096, sides)
out = torch.empty((4096, 4096), dtype=torch.uint8, device="cuda")
sweep = [int(a) for a in sys.argv[1:]] or [0]
for cb in sweep:
    eng.set_option("jpeg_chunk_bits", cb)
    eng.ingest_jpegs(blobs, (64, 64), "bgr", out=out)
    torch.cuda.synchronize()
    eng.timing_reset()
    best = 1e9
    for rep in range(4):
        t0 = time.perf_counter()
        packed = _pack_blobs(blobs)
        t1 = time.perf_counter()
        jpeg_info(blobs, _packed=packed)
        t2 = time.perf_counter()
        eng.ingest_jpegs(blobs, (64, 64), "bgr", out=out)
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        best = min(best, t3 - t2)
    ms, n = eng.timing_get("jpeg")
    print(f"chunk_bits {cb}: pack {1e3*(t1-t0):.2f} ms info {1e3*(t2-t1):.2f} ms ingest best {1e3*best:.2f} ms "
          f"({4096/best:.0f} faces/s)  jpeg device {ms / max(n, 1):.3f} ms/launch", flush=True)
