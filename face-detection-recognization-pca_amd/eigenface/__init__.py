"""eigenface — MI355X-native eigenfaces engine (fit + projection + nearest neighbour).

Drop-in for the PCA / recognition hot path of saladbkp/face-detection-recognization-PCA
(train-v4.py, scan-template-v4.py, useless/train.py, useless/scan.py), executed by
hand-written gfx950 HIP kernels in ``_lib/libeigenface.so`` (no CPU fallback).
"""
from ._native import EigenfaceError, NativeLibraryError, LIB_PATH  # noqa: F401
from .engine import Engine, FitResult, decode_keys, device_count, merge_matches_host  # noqa: F401
from .manual import ManualPCA, ManualStandardScaler, cosine_similarity, project_face_to_eigenspace  # noqa: F401
from .pca import (  # noqa: F401
    EigenfacePCA,
    get_engine,
    invalidate_uploads,
    set_resident_check,
    load_gallery_cache,
    manual_pca,
    recognize_face,
    recognize_face_dual_model,
    recognize_face_with_model,
    recognize_faces,
    recognize_faces_dual_model,
    save_gallery_cache,
)

__all__ = [
    "Engine", "FitResult", "decode_keys", "device_count", "EigenfacePCA", "get_engine",
    "invalidate_uploads", "set_resident_check", "manual_pca", "recognize_face", "recognize_face_with_model", "recognize_faces",
    "recognize_face_dual_model", "recognize_faces_dual_model", "merge_matches_host", "EigenfaceError",
    "NativeLibraryError", "LIB_PATH", "save_gallery_cache", "load_gallery_cache", "ManualPCA",
    "ManualStandardScaler", "project_face_to_eigenspace", "cosine_similarity",
]
