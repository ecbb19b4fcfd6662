"""Run the JPEG decoder's per-thread device functions in host loops (diagnostic build,
ef_diag_jpeg_decode_host) against Pillow's libjpeg-turbo on the test corpus — a CPU-only
check of decoder changes before they go to the GPU.  Needs `make -C
face-detection-recognization-pca_amd diag`."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "face-detection-recognization-pca_amd")]
import jpeg_cases as J  # noqa: E402
from eigenface.engine import _pack_blobs, jpeg_info  # noqa: E402

lib = C.CDLL(os.path.join(ROOT, "face-detection-recognization-pca_amd", "eigenface", "_lib", "libeigenface_diag.so"))
fn = lib.ef_diag_jpeg_decode_host
fn.argtypes = [C.c_void_p] * 3 + [C.c_int32, C.c_int32] + [C.c_void_p] * 3 + [C.c_int32, C.c_void_p]
bad = 0
cases = J.corpus()
CHUNK = int(sys.argv[1]) if len(sys.argv) > 1 else 0
for mode, mv, ch in (("bgr", 1, 3), ("gray", 0, 1)):
    blobs = [b for _, b in cases]
    data, offs, sizes, _keep = _pack_blobs(blobs)
    h, w, _, st = jpeg_info(blobs)
    px = h.astype(np.int64) * w * ch
    oo = np.zeros(len(blobs), np.int64)
    oo[1:] = np.cumsum(px)[:-1]
    out = np.zeros(int(px.sum()) + 1, np.uint8)
    st2 = np.zeros(len(blobs), np.int32)
    rounds = C.c_int32(0)
    fn(data, offs.ctypes.data, sizes.ctypes.data, len(blobs), mv, out.ctypes.data, oo.ctypes.data,
       st2.ctypes.data, CHUNK, C.byref(rounds))
    print(mode, "sync rounds", rounds.value)
    for i, (name, b) in enumerate(cases):
        ref = J.decode_ref(b, mode)
        got = out[oo[i]:oo[i] + px[i]].reshape(ref.shape)
        if not np.array_equal(got, ref):
            bad += 1
            d = np.abs(got.astype(int) - ref)
            print(mode, name, "max diff", d.max(), "n diff", int((d > 0).sum()), "of", d.size)
print("mismatches:", bad, "of", 2 * len(cases))
