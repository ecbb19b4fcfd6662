"""ctypes binding of libeigenface.so (include/eigenface.h).

The product path has no CPU fallback: if the HIP library is missing or cannot be
loaded, every entry point raises ``NativeLibraryError``.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib", "libeigenface.so")
# diagnostic builds (instrumented / ablated kernels, never a non-HIP fallback) by name
if os.environ.get("EF_LIB_VARIANT"):
    LIB_PATH = LIB_PATH.replace("libeigenface.so", f"libeigenface_{os.environ['EF_LIB_VARIANT']}.so")

EF_OK = 0
EF_U8, EF_F32, EF_F64 = 0, 1, 2
EF_METRIC_L2, EF_METRIC_COSINE = 0, 1
EF_FIT_STANDARDIZE = 0x1
EF_MODEL_BF16 = 0x2
EF_MEM_DEVICE = 0x100
EF_IMG_RGB = 0x200
EF_KERNEL_SEARCH, EF_KERNEL_PROJECT, EF_KERNEL_TMATCH, EF_KERNEL_INGEST, EF_KERNEL_HAAR, EF_KERNEL_JPEG, \
    EF_KERNEL_SYRK, EF_KERNEL_JPEG_HOST = 0, 1, 2, 3, 4, 5, 6, 7
EF_JPEG_GRAY, EF_JPEG_BGR = 0, 1
EF_JPEG_E_UNSUPPORTED, EF_JPEG_E_CORRUPT = -10, -11
EF_KEY_NONE = (1 << 63) - 1
EF_UNIQUE_ID_BYTES = 128
EF_OPT_FIT_MAX_ITERS, EF_OPT_FIT_FP32_COARSE, EF_OPT_COV_SLAB_BYTES, EF_OPT_TM_INT64_SUMS, EF_OPT_HAAR_ORDERED = \
    1, 2, 3, 4, 5
EF_OPT_JPEG_CHUNK_BITS = 6
EF_OPT_SEARCH_SPLIT_BF16 = 7
EF_OPT_JPEG_PART_FILES = 8
EF_OPT_FIT_CHEBYSHEV = 9
EF_OPT_HOST_THREADS = 10
EF_E_NUMERIC = -5


class ef_match(C.Structure):
    """include/eigenface.h ef_match: fp64 winner score, tie-tolerance scale, packed key."""
    _fields_ = [("score", C.c_double), ("scale", C.c_double), ("key", C.c_int64)]


# numpy view of an ef_match array
MATCH_DTYPE = [("score", "<f8"), ("scale", "<f8"), ("key", "<i8")]

_ERRNAMES = {-1: "EF_E_INVALID", -2: "EF_E_HIP", -3: "EF_E_STATE", -4: "EF_E_NOMEM", -5: "EF_E_NUMERIC"}


class NativeLibraryError(RuntimeError):
    """libeigenface.so is missing or unusable (there is no CPU fallback)."""


class EigenfaceError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{_ERRNAMES.get(code, code)}: {msg}")
        self.code = code


_lock = threading.Lock()
_lib = None

vp, i32, i64, u32 = C.c_void_p, C.c_int32, C.c_int64, C.c_uint32

_SIGS = {
    "ef_api_version": ([], C.c_int),
    "ef_device_count": ([C.POINTER(C.c_int)], C.c_int),
    "ef_create": ([C.c_int, C.POINTER(vp)], C.c_int),
    "ef_destroy": ([vp], None),
    "ef_last_error": ([vp], C.c_char_p),
    "ef_set_stream": ([vp, vp], C.c_int),
    "ef_use_own_stream": ([vp], C.c_int),
    "ef_get_stream": ([vp, C.POINTER(vp)], C.c_int),
    "ef_synchronize": ([vp], C.c_int),
    "ef_trim": ([vp], C.c_int),
    "ef_fit": ([vp, vp, i64, i64, i32, u32, vp, vp, vp, vp, vp, vp, vp, C.POINTER(i32), C.POINTER(i32)], C.c_int),
    "ef_fit_ex": ([vp, vp, i32, i64, i64, i32, u32, vp, vp, vp, vp, vp, vp, vp, C.POINTER(i32), C.POINTER(i32)],
                  C.c_int),
    "ef_colstats": ([vp, vp, i32, i64, i64, u32, vp, vp], C.c_int),
    "ef_chol_inv": ([vp, vp, i32, i64, C.c_double, vp, vp], C.c_int),
    "ef_fit_shard_stats": ([vp, vp, i64, i64, vp, vp, vp, u32], C.c_int),
    "ef_fit_from_stats": ([vp, vp, vp, vp, i64, i64, i32, u32, vp, vp, vp, vp, vp, vp, C.POINTER(i32),
                           C.POINTER(i32)], C.c_int),
    "ef_fit_transform": ([vp, vp, i64, i64, vp, vp, vp, i32, u32, vp], C.c_int),
    "ef_model_set": ([vp, vp, vp, i64, i32, u32], C.c_int),
    "ef_project": ([vp, vp, i32, i64, vp, u32], C.c_int),
    "ef_gallery_set": ([vp, vp, i64, i32, i64, u32], C.c_int),
    "ef_search": ([vp, vp, i64, i32, vp, u32], C.c_int),
    "ef_recognize": ([vp, vp, i32, i64, i32, vp, vp, u32], C.c_int),
    "ef_keys_decode": ([vp, i64, i32, vp, vp], None),
    "ef_search_schedule": ([i64, i32, i64, i32, vp, i32, C.POINTER(i32)], C.c_int),
    "ef_search_matches": ([vp, vp, i64, i32, vp, u32], C.c_int),
    "ef_recognize_matches": ([vp, vp, i32, i64, i32, vp, vp, u32], C.c_int),
    "ef_matches_merge": ([vp, vp, i32, i64, vp, vp, u32], C.c_int),
    "ef_comm_unique_id": ([vp], C.c_int),
    "ef_comm_init": ([vp, i32, i32, vp], C.c_int),
    "ef_comm_destroy": ([vp], C.c_int),
    "ef_comm_info": ([vp, C.POINTER(i32), C.POINTER(i32)], C.c_int),
    "ef_set_option": ([vp, i32, i64], C.c_int),
    "ef_get_option": ([vp, i32, C.POINTER(i64)], C.c_int),
    "ef_preprocess": ([vp, vp, vp, vp, vp, vp, i64, i32, i32, vp, u32], C.c_int),
    "ef_jpeg_info": ([vp, vp, vp, i32, vp, vp, vp, vp], C.c_int),
    "ef_jpeg_decode": ([vp, vp, vp, vp, i32, i32, vp, vp, vp, u32], C.c_int),
    "ef_jpeg_ingest": ([vp, vp, vp, vp, i32, i32, i32, i32, vp, vp, u32], C.c_int),
    "ef_tm_prepare": ([vp, vp, vp, vp, vp, i32, vp, vp, vp, i32, i32, i32, u32], C.c_int),
    "ef_tm_match": ([vp, vp, i64, vp, vp, vp, vp, u32], C.c_int),
    "ef_tm_info": ([vp, C.POINTER(i32), C.POINTER(i64), vp, vp], C.c_int),
    "ef_tm_sums_bits": ([i32, i32, i64], C.c_int),
    "ef_haar_set_cascade": ([vp, i32, i32, i32, vp, vp, i32, vp, vp, i32, vp, vp, vp, vp], C.c_int),
    "ef_haar_detect": ([vp, vp, i32, i32, i64, C.c_double, i32, i32, i32, i32, i32, vp, i32, C.POINTER(i32), vp, i32,
                        C.POINTER(i32), u32], C.c_int),
    "ef_timing_enable": ([vp, C.c_int], C.c_int),
    "ef_timing_get": ([vp, i32, C.POINTER(C.c_double), C.POINTER(i64)], C.c_int),
    "ef_timing_reset": ([vp], C.c_int),
}

EXPORTED_SYMBOLS = tuple(_SIGS)


def _load_torch_runtime_first():
    """One HIP runtime per process.  torch's wheel bundles its own ``libamdhip64.so``
    (soname ``libamdhip64.so.7``) and its libraries NEED it by the file name
    ``libamdhip64.so``; libeigenface NEEDs the soname.  Loaded after torch, libeigenface
    binds to torch's already-mapped runtime; loaded first, it maps /opt/rocm's and a later
    ``import torch`` maps a second runtime, and whichever initialises second sees no GPU
    (``ef_create`` fails with EF_E_HIP, or torch reports no device).  So torch, when it is
    installed, is imported before the library is opened."""
    import importlib.util
    import sys
    if "torch" in sys.modules or importlib.util.find_spec("torch") is None:
        return
    import torch  # noqa: F401


def lib():
    """Load (once) and return the ctypes handle; raise loudly when unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise NativeLibraryError(
                f"{LIB_PATH} not found: build it with `make -C face-detection-recognization-pca_amd` "
                "or __graft_entry__.build() (there is no CPU fallback)")
        _load_torch_runtime_first()
        try:
            h = C.CDLL(LIB_PATH)
        except OSError as e:  # pragma: no cover - depends on the box
            raise NativeLibraryError(f"cannot load {LIB_PATH}: {e}") from e
        for name, (args, res) in _SIGS.items():
            fn = getattr(h, name)
            fn.argtypes = args
            fn.restype = res
        if h.ef_api_version() != 7:
            raise NativeLibraryError("libeigenface.so API version mismatch")
        _lib = h
        return h


def check(ctx, rc):
    if rc != EF_OK:
        msg = lib().ef_last_error(ctx)
        raise EigenfaceError(rc, msg.decode() if msg else "")
    return rc
