"""JPEG ingest A/B over EF_OPT_JPEG_PART_FILES on bench.py's 4096-crop workload: wall
time per batch (device rows), device decode time, synchronisation rounds.
usage: python tools/jpeg_parts_ab.py [part sizes...]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "face-detection-recognization-pca_amd"))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from eigenface import Engine
    parts = [int(a) for a in sys.argv[1:]] or [8192, 2048, 1024]
    sides = [s for grp in bench.TEMPLATE_SIDES for s in grp]
    blobs = bench._face_jpegs(4096, sides)
    dev = torch.device("cuda", 0)
    out = torch.empty((len(blobs), 4096), dtype=torch.uint8, device=dev)
    eng = Engine(0)
    ref = None
    for rep in range(2):
        for p in parts:
            eng.set_option("jpeg_part_files", p)
            eng.ingest_jpegs(blobs, (64, 64), "bgr", out=out)
            torch.cuda.synchronize()
            eng.timing(True)
            eng.timing_reset()
            t = time.perf_counter()
            n = 10
            for _ in range(n):
                eng.ingest_jpegs(blobs, (64, 64), "bgr", out=out)
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t) / n
            k_ms, k_n = eng.timing_get("jpeg")
            eng.timing(False)
            rows = out.cpu()
            same = ref is None or torch.equal(rows, ref)
            ref = rows if ref is None else ref
            print(f"part_files={p}: {wall * 1e3:.3f} ms/batch = {len(blobs) / wall:.0f} faces/s, device decode "
                  f"{k_ms / n:.3f} ms in {k_n / n:.1f} launches, rows identical {same}", flush=True)
    eng.close()


if __name__ == "__main__":
    main()
