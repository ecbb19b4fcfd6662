"""Reference-surface mirror: the fit()/transform()/recognize() API and the drop-in
functions of the reference's hot path, all executed by libeigenface on the GPU.

* ``manual_pca``                 — useless/train.py:56-128
* ``EigenfacePCA``               — FaceTrainer.train_pca_model's StandardScaler+PCA
                                   (train-v4.py:110-146) and sklearn's
                                   fit/transform/fit_transform surface
* ``recognize_face_with_model``  — scan-template-v4.py:270-287
* ``recognize_face``             — useless/scan.py:100-132
* ``save_gallery_cache`` / ``load_gallery_cache`` — raw ``.npy`` gallery features
"""
from __future__ import annotations

import os
import threading

import numpy as np

from .engine import Engine

_engines: dict[tuple[int, str], Engine] = {}
_elock = threading.Lock()


def get_engine(device: int = 0, pool: str = "shared") -> Engine:
    """Process-wide Engine for a device (created on first use).  ``pool`` names separate
    engines on one device: the manual helpers (``eigenface.manual``) keep their one-off
    models and one-row galleries on their own engine, so they never evict the model and
    gallery that the recognise functions keep resident on the shared one."""
    with _elock:
        e = _engines.get((device, pool))
        if e is None:
            e = Engine(device)
            _engines[(device, pool)] = e
        return e


def _as_pixels(X):
    """Fit input: uint8 pixels (train-v4.py:68,73) go to the exact integer kernels, and so
    do float arrays holding integral 0..255 values (useless/train.py:40 flattens the uint8
    pixels to float64) — same numbers, exact products.  Any other float data (e.g.
    standardised faces, scripts/manual/train-v2.py:194-197) is fitted as float64 on the
    fp64 GEMM path (ef_fit_ex)."""
    x = np.asarray(X)
    if x.dtype == np.uint8:
        return x
    if x.dtype == np.float32 and not np.all(np.isfinite(x)):
        raise ValueError("fit input contains NaN or inf")
    xf = np.asarray(x, dtype=np.float64)
    if not np.all(np.isfinite(xf)):
        raise ValueError("fit input contains NaN or inf")
    xu = np.clip(np.rint(xf), 0, 255)
    if np.array_equal(xu, xf):
        return xu.astype(np.uint8)
    return x if x.dtype == np.float32 else xf


class EigenfacePCA:
    """Eigenfaces estimator with sklearn-compatible attributes.

    ``standardize=True`` reproduces train-v4.py's ``StandardScaler`` -> ``PCA``
    (with the deterministic full solver); ``standardize=False`` is manual_pca.
    After ``fit`` the recognition model (folded into ``(p - mu_f) . W``) and the
    training features (as gallery) are resident on the GPU.
    """

    def __init__(self, n_components=50, standardize=False, device=0):
        self.n_components = n_components
        self.standardize = standardize
        self.device = device

    # -------------------------------------------------------------------- fit
    def fit(self, X, y=None):
        x = _as_pixels(X)
        n, d = x.shape
        eng = get_engine(self.device)
        r = eng.fit(x, self.n_components, standardize=self.standardize)
        k = r.k
        self.n_samples_, self.n_features_in_ = n, d
        self.n_components_ = k
        self.mean_face_ = r.mean
        self.components_ = r.components
        self.explained_variance_ = r.eigenvalues
        self.total_var_ = r.total_var
        self.explained_variance_ratio_ = r.eigenvalues / r.total_var
        self.singular_values_ = np.sqrt(np.maximum(r.eigenvalues, 0.0) * (n - 1))
        rank = min(n, d)
        self.noise_variance_ = float((r.total_var - r.eigenvalues.sum()) / (rank - k)) if k < rank else 0.0
        if self.standardize:
            self.scaler_mean_, self.scaler_var_, self.scaler_scale_ = r.mean, r.var, r.scale
            self.mean_ = np.zeros(d)  # PCA mean of standardised data (exactly 0)
            w = (r.components / r.scale[None, :]).T
        else:
            self.scaler_mean_ = self.scaler_var_ = self.scaler_scale_ = None
            self.mean_ = r.mean
            w = r.components.T
        self.face_features_ = r.projection
        self.fit_iters_ = r.iters
        self._W = np.ascontiguousarray(w, dtype=np.float32)
        self._mu = np.ascontiguousarray(r.mean, dtype=np.float32)
        # owner tokens: the engine's resident model / gallery are ours only while the
        # engine still carries these exact tokens (another estimator or a drop-in function
        # may have replaced them in between)
        self._model_token = object()
        self._gallery_token = None
        self._gallery_src = None
        return self

    def fit_transform(self, X, y=None):
        return self.fit(X).face_features_

    # --------------------------------------------------------------- transform
    def _ensure_model(self, eng):
        if eng.model_owner is not self._model_token:
            eng.set_model(self._mu, self._W, owner=self._model_token)

    def transform(self, X):
        """(p - mean) . W on the GPU (fp32 MFMA), returned as float64."""
        eng = get_engine(self.device)
        self._ensure_model(eng)
        x = np.asarray(X)
        if x.dtype != np.uint8:
            x = np.asarray(x, dtype=np.float32)
        return eng.project(x).astype(np.float64)

    # --------------------------------------------------------------- recognize
    def set_gallery(self, features=None):
        """Gallery rows for ``recognize`` (default: the training features); a path loads a
        raw ``.npy`` feature cache (memory-mapped, see ``save_gallery_cache``)."""
        eng = get_engine(self.device)
        if isinstance(features, (str, os.PathLike)):
            features = load_gallery_cache(features)
        self._gallery_src = self.face_features_ if features is None else np.asarray(features)
        self._gallery_token = object()
        eng.set_gallery(np.asarray(self._gallery_src, dtype=np.float32), owner=self._gallery_token)
        return self

    def save_gallery(self, path):
        """Write the current gallery (default: the training features) as a raw ``.npy``
        cache, so a large gallery is reloaded instead of re-projected."""
        save_gallery_cache(path, self.face_features_ if self._gallery_src is None else self._gallery_src)
        return path

    def recognize(self, P, metric="cosine", threshold=None):
        """Batched recognise: returns (idx, score); with ``threshold`` (cosine
        only) idx is -1 where score < threshold (scan-template-v4.py:278)."""
        eng = get_engine(self.device)
        self._ensure_model(eng)
        if self._gallery_token is None:
            self.set_gallery()
        elif eng.gallery_owner is not self._gallery_token:  # replaced by someone else: re-upload
            eng.set_gallery(np.asarray(self._gallery_src, dtype=np.float32), owner=self._gallery_token)
        idx, best = eng.recognize(P, metric)
        if threshold is not None:
            idx = np.where(best >= threshold, idx, -1)
        return idx, best


def save_gallery_cache(path, features):
    """Gallery features as a raw float32 ``.npy`` file (SURVEY §5 checkpoint/resume: the 1M
    gallery is not re-projected on restart).  Plain array data, no pickle."""
    np.save(path, np.ascontiguousarray(features, dtype=np.float32), allow_pickle=False)


def load_gallery_cache(path, mmap=True):
    """The cache written by ``save_gallery_cache``: a read-only memory map by default, which
    ``Engine.set_gallery`` uploads without an extra host copy."""
    a = np.load(path, mmap_mode="r" if mmap else None, allow_pickle=False)
    if a.ndim != 2 or a.dtype != np.float32:
        raise ValueError(f"{path}: expected a 2-D float32 feature array, got {a.dtype} {a.shape}")
    return a


def manual_pca(data_matrix, n_components=None, device=0):
    """Drop-in for manual_pca (useless/train.py:56-128), computed on the GPU.

    Returns ``(eigenfaces (d,k), mean_face (d,), projected_data (n,k),
    eigenvalues (k,))`` float64.  Eigenvector signs follow sklearn's svd_flip
    rule (the reference's LAPACK signs are arbitrary)."""
    x = _as_pixels(data_matrix)
    n, d = x.shape
    if n_components is None:
        n_components = min(n - 1, d)
    r = get_engine(device).fit(x, n_components, standardize=False)
    # (d, k) Fortran-ordered like the reference's faces[:, order][:, :k] (the layout of
    # the committed models/*_pca_model.pkl)
    return r.components.T, r.mean, r.projection, r.eigenvalues


# ------------------------------------------------------------------ recognize
class _ArrayToken:
    """Owner token of an uploaded host array: the array itself (kept alive, so its id
    cannot be reused), its data pointer, shape and dtype, plus a digest of ALL its bytes,
    so an in-place edit anywhere (re-enrolling one person's row of a large gallery) makes
    the next call re-upload — the reference reads the array it is given on every call.
    The digest is xxh3-128 (~20 GB/s on one host core: a 1M x 128 fp32 gallery costs
    ~25 ms, half of what its re-upload over PCIe would; the 2 GB C5 gallery ~100 ms),
    blake2b (seconds per GB) where xxhash is absent.  It is paid on EVERY recognise call,
    which dominates single-face calls on large galleries: a caller that never edits its
    arrays in place can switch it off with ``set_resident_check("identity")`` (same
    object, pointer, shape and dtype only) and call :func:`invalidate_uploads` after any
    edit."""

    def __init__(self, a):
        self.a = a
        self.ptr = a.__array_interface__["data"][0]
        self.shape, self.dtype = a.shape, a.dtype
        self.digest = _digest(a) if _RESIDENT_CHECK == "digest" else None

    def matches(self, a):
        if not (a is self.a and a.shape == self.shape and a.dtype == self.dtype
                and a.__array_interface__["data"][0] == self.ptr):
            return False
        if _RESIDENT_CHECK != "digest":
            return True
        if self.digest is None:  # token made while the check was off: digest it now
            self.digest = _digest(a)
            return False
        return _digest(a) == self.digest


_RESIDENT_CHECK = "digest"


def set_resident_check(mode: str):
    """How the recognise helpers decide that a resident gallery / model is still the host
    array they are given: "digest" (default: a full xxh3-128 hash of its bytes per call,
    so in-place edits re-upload) or "identity" (the same array object, pointer, shape and
    dtype — no per-call hashing; the caller promises not to edit resident arrays in place
    or calls invalidate_uploads after doing so)."""
    global _RESIDENT_CHECK
    if mode not in ("digest", "identity"):
        raise ValueError("mode must be 'digest' or 'identity'")
    _RESIDENT_CHECK = mode


try:
    import xxhash as _xxhash
except ImportError:  # pragma: no cover - the image ships xxhash
    _xxhash = None


def _digest(a):
    b = np.ascontiguousarray(a).view(np.uint8).reshape(-1)
    if _xxhash is not None:
        return _xxhash.xxh3_128_digest(b)
    import hashlib
    return hashlib.blake2b(b, digest_size=16).digest()


def invalidate_uploads(device: int = 0):
    """Forget which host arrays the device's resident models and galleries came from: the
    next recognise call re-uploads them (the digest already catches in-place edits; this
    is for arrays changed behind numpy's back, e.g. by a foreign buffer writer)."""
    for (dev, _pool), eng in list(_engines.items()):
        if dev == device:
            eng.model_owner = None
            eng.gallery_owner = None


def _gallery_engine(features, device, pool="shared"):
    """Engine whose resident gallery holds ``features`` (uploaded when the engine's owner
    token is not this array's token)."""
    eng = get_engine(device, pool)
    a = features if isinstance(features, np.ndarray) else np.asarray(features)
    tok = eng.gallery_owner
    if not (isinstance(tok, _ArrayToken) and tok.matches(a)):
        eng.set_gallery(np.asarray(a, dtype=np.float32), owner=_ArrayToken(a))
    return eng


def _model_engine(mean, W, device, pool="shared"):
    """Engine whose resident model is (mean, W) (same owner-token rule)."""
    eng = get_engine(device, pool)
    tok = eng.model_owner
    if not (isinstance(tok, tuple) and len(tok) == 2 and tok[0].matches(mean) and tok[1].matches(W)):
        eng.set_model(np.asarray(mean, dtype=np.float32), np.asarray(W, dtype=np.float32),
                      owner=(_ArrayToken(mean), _ArrayToken(W)))
    return eng


def recognize_face_with_model(face_features, model_data, threshold=0.7, device=0):
    """Drop-in for ``recognize_face_with_model`` (scan-template-v4.py:270-287):
    cosine vs ``model_data['face_features']`` on the GPU, first argmax,
    ``>= threshold``, label via ``face_labels`` / ``person_id_map``."""
    eng = _gallery_engine(model_data["face_features"], device)
    idx, best = eng.search(np.asarray(face_features, dtype=np.float32).reshape(1, -1), "cosine")
    i, sim = int(idx[0]), float(best[0])
    if i >= 0 and sim >= threshold:
        pid = model_data["face_labels"][i]
        name = "unknown"
        for nm, v in model_data["person_id_map"].items():
            if v == pid:
                name = nm
                break
        return pid, name, sim
    return -1, "unknown", sim


def recognize_face(face_vector, model_data, similarity_threshold=0.7, device=0):
    """Drop-in for ``recognize_face`` on a ``models/*_pca_model.pkl`` dict
    (useless/scan.py:100-132): returns ``(person_name, max_similarity,
    is_recognized)``."""
    return recognize_faces(np.asarray(face_vector).reshape(1, -1), model_data, similarity_threshold, device)[0]


def recognize_faces(face_vectors, model_data, similarity_threshold=0.7, device=0):
    """Batched ``recognize_face``: one GPU projection + cosine arg-best for all rows of
    ``face_vectors`` (b, d) — the loop useless/scan.py:168-215 runs per detection.
    Each call hashes the model's and gallery's host arrays to decide whether the resident
    copies are current (``_ArrayToken``; ~25 ms per 512 MB): see set_resident_check."""
    mean, ef = _as_array(model_data["mean_face"]), _as_array(model_data["eigenfaces"])
    eng = _model_engine(mean, ef, device)
    _gallery_engine(_as_array(model_data["projected_data"]), device)
    p = np.asarray(face_vectors)
    p = p if p.dtype == np.uint8 else p.astype(np.float32)
    _, best = eng.recognize(p, "cosine")
    name = model_data["person_name"]
    return [(name, float(s), bool(s >= similarity_threshold)) for s in best]


def recognize_face_dual_model(face_vector, dark_model_data, light_model_data, similarity_threshold=0.7, device=0):
    """Drop-in for ``recognize_face_dual_model`` (useless/scan.py:134-166): the face is
    recognised by the dark and the light model, OR-combined; the confidence is the
    larger similarity and the name comes from the dark model on ties (``>=``).  Returns
    ``(person_name, best_confidence, is_recognized, dark_similarity, light_similarity)``."""
    return recognize_faces_dual_model(np.asarray(face_vector).reshape(1, -1), dark_model_data, light_model_data,
                                      similarity_threshold, device)[0]


def recognize_faces_dual_model(face_vectors, dark_model_data, light_model_data, similarity_threshold=0.7, device=0):
    """Batched :func:`recognize_face_dual_model`: one GPU pass per model over all rows."""
    dark = recognize_faces(face_vectors, dark_model_data, similarity_threshold, device)
    light = recognize_faces(face_vectors, light_model_data, similarity_threshold, device)
    out = []
    for (dn, ds, dr), (ln, ls, lr) in zip(dark, light):
        out.append((dn if ds >= ls else ln, max(ds, ls), dr or lr, ds, ls))
    return out


def _as_array(a):
    return a if isinstance(a, np.ndarray) else np.asarray(a)
