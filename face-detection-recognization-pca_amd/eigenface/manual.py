"""The reference's "manual" (no-sklearn) surface, computed by libeigenface:

* ``ManualPCA``            — scripts/manual/train-v2.py:9-51 (fit / transform / fit_transform)
* ``ManualStandardScaler`` — scripts/manual/train-v2.py:53-72
* ``project_face_to_eigenspace`` — useless/scan.py:80-98
* ``cosine_similarity``    — useless/scan.py:58-78 (vector . vector)

ManualPCA's fit accepts what the manual trainer feeds it: the scaler's float64 output
(train-v2.py:194-197), fitted on the GPU by ``ef_fit_ex`` (fp64 column statistics, Gram or
covariance on the fp64 MFMA GEMM with centring in the operand loads, eigensolve,
back-projection); uint8 / integral pixel input takes the exact integer kernels.
Differences from the reference, both inside its own arbitrariness:
eigenvector signs follow sklearn's svd_flip rule (``np.linalg.eigh``'s are LAPACK's
choice), and with fewer samples than pixels the top components come from the Gram
matrix (same eigenpairs as ``np.cov``'s d x d matrix; at most n of them are produced).
"""
from __future__ import annotations

import numpy as np

from .pca import _as_pixels, _gallery_engine, _model_engine, get_engine


class ManualStandardScaler:
    """scripts/manual/train-v2.py:53-72: ``mean_ = np.mean(X, 0)``, ``scale_ = np.std(X, 0)``
    (ddof 0) with exact zeros replaced by 1; ``transform = (X - mean_) / scale_``.
    The statistics come from ``ef_colstats`` (exact integer sums for uint8 pixels,
    two-pass fp64 otherwise); ``transform`` is the reference's elementwise host expression,
    returning float64 like it."""

    def __init__(self, device=0):
        self.mean_ = None
        self.scale_ = None
        self.device = device

    def fit(self, X):
        mean, var = get_engine(self.device).colstats(np.asarray(X))
        self.mean_ = mean
        scale = np.sqrt(var)
        scale[scale == 0] = 1  # train-v2.py:62-63 (exact zeros only, unlike sklearn's rule)
        self.scale_ = scale
        return self

    def transform(self, X):
        return (np.asarray(X, dtype=np.float64) - self.mean_) / self.scale_

    def fit_transform(self, X):
        return self.fit(X).transform(X)


class ManualPCA:
    """scripts/manual/train-v2.py:9-51 on the GPU.  After ``fit``: ``mean_`` (d,),
    ``components_`` (k, d) (top eigenvectors of the covariance as rows, descending),
    ``explained_variance_ratio_`` = λ_i / Σ all eigenvalues (= λ_i / trace, :38-40), plus
    ``explained_variance_`` (the λ_i) and ``n_components_``."""

    def __init__(self, n_components=50, device=0):
        self.n_components = n_components
        self.components_ = None
        self.mean_ = None
        self.explained_variance_ratio_ = None
        self.device = device
        self._train = None

    def fit(self, X):
        x = _as_pixels(X)
        r = get_engine(self.device).fit(x, self.n_components, standardize=False, projection=True)
        self.mean_ = r.mean
        self.components_ = r.components
        self.explained_variance_ = r.eigenvalues
        self.n_components_ = r.k
        self.explained_variance_ratio_ = r.eigenvalues / r.total_var if r.total_var > 0 else np.zeros(r.k)
        self._train = (x, r.projection)  # fit_transform's output, already computed in fp64
        self._folded = None
        return self

    def transform(self, X):
        """``(X - mean_) . components_ᵀ`` (train-v2.py:44-47): the GPU projection (fp32 MFMA,
        input uint8 or float32), returned as float64."""
        if self.components_ is None:
            raise RuntimeError("ManualPCA is not fitted")
        if self._folded is None:
            self._folded = (np.ascontiguousarray(self.mean_, dtype=np.float32),
                            np.ascontiguousarray(self.components_.T, dtype=np.float32))
        eng = _model_engine(self._folded[0], self._folded[1], self.device, "manual")
        x = np.asarray(X)
        x = x if x.dtype == np.uint8 else np.asarray(x, dtype=np.float32)
        return eng.project(np.atleast_2d(x)).astype(np.float64)

    def fit_transform(self, X):
        """``fit(X).transform(X)`` (:49-51): the fit's own fp64 training projection."""
        return self.fit(X)._train[1]


def project_face_to_eigenspace(face_vector, eigenfaces, mean_face, device=0):
    """useless/scan.py:80-98: ``(face_vector - mean_face) . eigenfaces`` with
    ``eigenfaces`` (d, k) as stored in models/*_pca_model.pkl.  One face (d,) -> (k,), or
    a batch (b, d) -> (b, k), float64; computed by the GPU projection (fp32 MFMA)."""
    ef = np.asarray(eigenfaces)
    mu = np.asarray(mean_face)
    eng = _model_engine(mu, ef, device, "manual")
    v = np.asarray(face_vector)
    p = v if v.dtype == np.uint8 else np.asarray(v, dtype=np.float32)
    f = eng.project(np.atleast_2d(p)).astype(np.float64)
    return f[0] if v.ndim == 1 else f


def cosine_similarity(vec1, vec2, device=0):
    """useless/scan.py:58-78: ``vec1 . vec2 / (|vec1| |vec2|)``, 0.0 when either norm is
    0, for vectors of any length up to 65536.  The product is scored by the GPU search (a
    one-row gallery; the match record's score is the fp64 similarity of the fp32 inputs),
    on the helpers' own engine, so it never evicts a resident recognition gallery.  One
    call is one GPU round trip: to score a face against a whole gallery (the loop of
    useless/scan.py:122-124) call ``recognize_faces`` / ``Engine.search`` once instead."""
    a = np.asarray(vec1, dtype=np.float64).ravel()
    b = np.asarray(vec2, dtype=np.float64).ravel()
    if a.shape != b.shape:
        raise ValueError(f"vectors differ in length: {a.shape[0]} vs {b.shape[0]}")
    if np.linalg.norm(a) == 0 or np.linalg.norm(b) == 0:  # :70-74
        return 0.0
    g = np.ascontiguousarray(b[None, :], dtype=np.float32)
    eng = _gallery_engine(g, device, "manual")
    m = eng.search_matches(np.ascontiguousarray(a[None, :], dtype=np.float32), "cosine")
    return float(-m["score"][0])
