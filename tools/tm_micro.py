"""Template-localiser efficiency by shape: uniform problem sets whose result maps are whole
128 x 128 tiles, sized to whole rounds of 256 workgroups; ideal = every SIMD issuing 2
waves x 2*NKB MFMAs (32 cycles each) per template row.  Prints device ms per frame for the
tm_* kernels (hipEvents) and the tm_corr share from a second, corr-only estimate."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "face-detection-recognization-pca_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from eigenface import Engine  # noqa: E402

torch.cuda.set_device(0)
eng = Engine(0)
eng.timing(True)
rng = np.random.default_rng(0)
H, W = 480, 640
frame = rng.integers(0, 256, (H, W), dtype=np.uint8)
out = []
for th, tw in [(97, 1), (97, 129), (97, 257), (225, 129), (33, 129), (97, 65), (97, 193)]:
    hr, wr = H - th + 1, W - tw + 1
    tiles = (hr + 127) // 128 * ((wr + 127) // 128) * ((th + 127) // 128)
    nprob = max(1, 768 // tiles)
    t = rng.integers(0, 256, (th, tw), dtype=np.uint8)
    eng.tm_prepare([t], [(0, th, tw)] * nprob, (H, W))
    eng.tm_match(frame)
    eng.timing_reset()
    for _ in range(10):
        eng.tm_match(frame)
    ms, n = eng.timing_get("tmatch")
    ms /= max(n, 1)
    nkb = (min(tw, 352) + 62) // 32
    items = tiles * nprob
    rounds = -(-items // 256)
    ideal_cycles = rounds * min(th, 128) * 2 * 2 * nkb * 32 * (th + 127) // 128 / ((th + 127) // 128)
    rec = {"th": th, "tw": tw, "nkb": nkb, "hr": hr, "wr": wr, "items": items, "ms": round(ms, 4),
           "ideal_ms_2.1GHz": round(ideal_cycles / 2.1e9 * 1e3, 4)}
    out.append(rec)
    print(json.dumps(rec), flush=True)
eng.close()
