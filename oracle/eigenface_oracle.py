"""CPU oracle for the eigenfaces hot path — TEST INFRASTRUCTURE ONLY.

This module is a plain NumPy restatement of the reference algorithm
(saladbkp/face-detection-recognization-PCA, snapshot 2025-08-29).  It exists
to *check* the MI355X path, never to stand in for it:

  * only ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg
    of ``bench.py`` may import it;
  * the product package (``face-detection-recognization-pca_amd/eigenface``)
    never imports it and fails loudly when its HIP library is missing.

Parity pinning (see ``tests/golden/make_goldens.py`` and DESIGN.md §Oracle):
the reference's own Python functions were imported in the build container and
run on the reference's committed faces / synthetic inputs; their outputs are
committed as ``tests/golden/*.npz`` and this restatement is checked against
them (``tests/test_oracle_golden.py``).  The explained-variance ratios written
by the reference into ``models/Joseph_Lai_{light,dark}_model_info.json`` pin
the real-data fit end to end.

Every function cites the reference file:line it restates.
"""
from __future__ import annotations

import numpy as np

__all__ = [
    "manual_pca",
    "standard_scaler_fit",
    "pca_full_fit",
    "train_pca_model",
    "sklearn_transform",
    "fold_projection",
    "project",
    "cosine_scores",
    "cosine_argmax",
    "l2_argmin",
    "recognize_face_with_model",
    "recognize_face_manual",
    "manual_model_info_evr",
    "synth_faces",
    "int_synth_faces",
    "pca_cov_fit",
    "synth_basis",
    "synth_mean_face",
    "planted_probes",
    "manual_standard_scaler",
    "manual_pca_cov",
    "cosine_similarity_vec",
]


# --------------------------------------------------------------------------
# Fit: manual Gram-trick PCA  (useless/train.py:56-128)
# --------------------------------------------------------------------------
def manual_pca(data_matrix, n_components=None):
    """Restates ``manual_pca`` (useless/train.py:56-128).

    mean (:70) -> centre (:74) -> Gram A.A^T/(n-1) when n<d (:82-85) or the
    d x d covariance otherwise (:97-103) -> ``eigh`` (:88) -> back-project
    A^T.V (:91) -> unit columns (:94-95) -> descending order (:106-108) ->
    keep k (:111-116) -> project A.E (:122).

    Returns ``(eigenfaces (d,k), mean_face (d,), projected (n,k),
    eigenvalues (k,))`` in float64, exactly the reference's tuple.
    """
    x = np.asarray(data_matrix, dtype=np.float64)
    n, d = x.shape
    mu = x.mean(axis=0)
    a = x - mu
    if n < d:
        gram = (a @ a.T) / (n - 1)
        lam, vecs = np.linalg.eigh(gram)
        faces = a.T @ vecs
        faces = faces / np.linalg.norm(faces, axis=0, keepdims=True)
    else:
        cov = np.cov(a.T)
        lam, faces = np.linalg.eigh(cov)
    order = np.argsort(lam)[::-1]
    lam = lam[order]
    faces = faces[:, order]
    if n_components is None:
        n_components = min(n - 1, d)
    k = min(n_components, lam.shape[0])
    lam = lam[:k]
    faces = faces[:, :k]
    return faces, mu, a @ faces, lam


def manual_model_info_evr(eigenvalues):
    """``explained_variance_ratio`` field of ``*_model_info.json``.

    useless/train.py:182 divides by the sum of the *kept* k eigenvalues and
    keeps the first 10 entries.
    """
    lam = np.asarray(eigenvalues, dtype=np.float64)
    return (lam / lam.sum())[:10]


# --------------------------------------------------------------------------
# Fit: the "manual" trainer's classes (scripts/manual/train-v2.py:9-72)
# --------------------------------------------------------------------------
def manual_standard_scaler(x):
    """``ManualStandardScaler.fit_transform`` (scripts/manual/train-v2.py:58-72):
    ``mean = np.mean(X, 0)``, ``scale = np.std(X, 0)`` with exact zeros set to 1,
    ``Z = (X - mean) / scale``.  Returns ``(Z, mean, scale)`` float64."""
    x = np.asarray(x, dtype=np.float64)
    mean = np.mean(x, axis=0)
    scale = np.std(x, axis=0)
    scale[scale == 0] = 1
    return (x - mean) / scale, mean, scale


def manual_pca_cov(x, n_components):
    """``ManualPCA.fit`` + ``transform`` (scripts/manual/train-v2.py:16-47): mean (:19),
    centre (:22), the full d x d ``np.cov`` (:25), ``eigh`` (:28), descending (:31-33),
    top-k rows (:36), ratio over the sum of ALL eigenvalues (:39-40); features
    ``(X - mean) . components^T``.  Eigenvector signs are normalised to sklearn's
    svd_flip rule (largest-|.| entry positive) since eigh's are arbitrary.  Returns
    ``(components (k, d), mean, evr (k,), eigenvalues (k,), features (n, k))``."""
    x = np.asarray(x, dtype=np.float64)
    mean = np.mean(x, axis=0)
    xc = x - mean
    lam, vec = np.linalg.eigh(np.cov(xc.T))
    order = np.argsort(lam)[::-1]
    lam, vec = lam[order], vec[:, order]
    comps, _ = _svd_flip_rows(vec[:, :n_components].T)
    evr = lam[:n_components] / np.sum(lam)
    return comps, mean, evr, lam[:n_components], xc @ comps.T


def cosine_similarity_vec(v1, v2):
    """useless/scan.py:58-78 for two vectors (0.0 when a norm is 0)."""
    a, b = np.asarray(v1, dtype=np.float64), np.asarray(v2, dtype=np.float64)
    na, nb = np.linalg.norm(a), np.linalg.norm(b)
    if na == 0 or nb == 0:
        return 0.0
    return float(np.dot(a, b) / (na * nb))


# --------------------------------------------------------------------------
# Fit: sklearn path used by train-v4.py:126-146
# --------------------------------------------------------------------------
def standard_scaler_fit(x):
    """``StandardScaler().fit`` as called at train-v4.py:131.

    Semantics of sklearn 1.7 ``_data.py:1040-1051``: population variance
    (ddof 0) in float64; features whose variance is within the two-pass
    error bound of zero (``_is_constant_feature`` ``_data.py:76-89``) get
    scale 1.  Returns ``(mean, var, scale)``.
    """
    x = np.asarray(x, dtype=np.float64)
    n = x.shape[0]
    mean = x.mean(axis=0)
    var = ((x - mean) ** 2).mean(axis=0)
    eps = np.finfo(np.float64).eps
    constant = var <= n * eps * var + (n * mean * eps) ** 2
    scale = np.sqrt(var)
    scale[constant] = 1.0
    return mean, var, scale


def _svd_flip_rows(vt):
    """sklearn ``svd_flip(u_based_decision=False)`` (extmath.py:944-952):
    the largest-|.| entry (first on ties) of every row is made positive."""
    pos = np.argmax(np.abs(vt), axis=1)
    signs = np.sign(vt[np.arange(vt.shape[0]), pos])
    signs[signs == 0] = 1.0
    return vt * signs[:, None], signs


def pca_full_fit(z, n_components):
    """``PCA(n_components, svd_solver='full').fit`` (sklearn _pca.py:537-700).

    Returns a dict with the attributes ``transform``/``fit_transform`` need:
    ``mean_, components_, explained_variance_, explained_variance_ratio_,
    singular_values_, noise_variance_, n_components_, n_samples_`` plus the
    ``fit_transform`` output ``U*S`` (_pca.py:466-477).
    """
    z = np.asarray(z, dtype=np.float64)
    n, d = z.shape
    k = int(n_components)
    if not 0 <= k <= min(n, d):
        raise ValueError("n_components must be between 0 and min(n_samples, n_features)")
    mean = z.mean(axis=0)
    zc = z - mean
    u, s, vt = np.linalg.svd(zc, full_matrices=False)
    vt, signs = _svd_flip_rows(vt)
    u = u * signs[None, :]
    ev = s ** 2 / (n - 1)
    total = ev.sum()
    noise = ev[k:].mean() if k < min(n, d) else 0.0
    return {
        "mean_": mean,
        "components_": vt[:k].copy(),
        "explained_variance_": ev[:k].copy(),
        "explained_variance_ratio_": (ev / total)[:k].copy(),
        "singular_values_": s[:k].copy(),
        "noise_variance_": float(noise),
        "n_components_": k,
        "n_samples_": n,
        "total_var": float(total),
        "fit_transform": u[:, :k] * s[:k],
    }


def pca_cov_fit(x, n_components, standardize=True, chunk=2048):
    """``train_pca_model``'s StandardScaler + PCA for n >= d through the covariance
    branch of manual_pca (useless/train.py:97-103: ``np.cov`` + ``eigh``) instead of
    an SVD of the n x d matrix — the same estimator (``components_`` = top
    eigenvectors of the covariance of the standardised data, ``explained_variance_``
    = its eigenvalues, sklearn's svd_flip sign rule, extmath.py:946-952), affordable
    at the C3 shape (d = 16384).  Only the top ``n_components`` pairs are computed
    (LAPACK dsyevr through scipy).  Returns the dict of :func:`pca_full_fit` plus
    ``scaler``.  The three phases are separate functions (cov_standardised,
    top_eigh, project_standardised) so a CPU baseline can time them apart."""
    k = int(n_components)
    st = cov_standardised(x, standardize, chunk)
    lam, vt = top_eigh(st["cov"], k)
    del st["cov"]
    feats = project_standardised(x, st, vt, chunk)
    total = st["total_var"]
    return {
        "scaler": (st["s_mean"], st["s_var"], st["s_scale"]),
        "mean_": st["zmean"],
        "components_": vt,
        "explained_variance_": lam,
        "explained_variance_ratio_": lam / total,
        "total_var": total,
        "fit_transform": feats,
    }


def cov_standardised(x, standardize=True, chunk=2048):
    """Phase 1 of :func:`pca_cov_fit`: StandardScaler statistics, then the fp64
    covariance of the standardised data (PCA centres z again: _pca.py:741-743)."""
    x = np.asarray(x)
    n, d = x.shape
    if standardize:
        s_mean, s_var, s_scale = standard_scaler_fit(x)
    else:
        s_mean = x.astype(np.float64).mean(axis=0)
        s_var = s_scale = np.ones(d)
    zmean = np.zeros(d)
    for a in range(0, n, chunk):
        zmean += ((x[a:a + chunk].astype(np.float64) - s_mean) / s_scale).sum(axis=0)
    zmean /= n
    cov = np.zeros((d, d))
    for a in range(0, n, chunk):
        zc = (x[a:a + chunk].astype(np.float64) - s_mean) / s_scale - zmean
        cov += zc.T @ zc
    cov /= n - 1
    return {"s_mean": s_mean, "s_var": s_var, "s_scale": s_scale, "zmean": zmean, "cov": cov,
            "total_var": float(np.trace(cov))}


def top_eigh(cov, k, overwrite=True):
    """Phase 2: the top k eigenpairs (LAPACK dsyevr), descending, svd_flip signs.
    Returns (eigenvalues, components as rows)."""
    import scipy.linalg as sla
    d = cov.shape[0]
    lam, vec = sla.eigh(cov, subset_by_index=[d - k, d - 1], driver="evr", overwrite_a=overwrite)
    order = np.argsort(lam)[::-1]
    vt, _ = _svd_flip_rows(vec[:, order].T)
    return lam[order], vt


def project_standardised(x, st, vt, chunk=2048):
    """Phase 3: the training projection of the standardised, re-centred data."""
    x = np.asarray(x)
    feats = np.empty((x.shape[0], vt.shape[0]))
    for a in range(0, x.shape[0], chunk):
        feats[a:a + chunk] = ((x[a:a + chunk].astype(np.float64) - st["s_mean"]) / st["s_scale"]
                              - st["zmean"]) @ vt.T
    return feats


def train_pca_model(face_images, n_components):
    """``FaceTrainer.train_pca_model`` (train-v4.py:110-146) with the PCA
    solver pinned to ``full`` (the reference's ``auto`` picks the unseeded
    randomized solver).

    Returns ``dict(mean_face, scaler=(mean, var, scale), pca=<pca_full_fit>,
    face_features, eigenfaces)``.
    """
    x = np.asarray(face_images)
    mean_face = x.astype(np.float64).mean(axis=0)            # :127
    s_mean, s_var, s_scale = standard_scaler_fit(x)          # :131
    z = (x.astype(np.float64) - s_mean) / s_scale
    pca = pca_full_fit(z, n_components)                      # :134
    return {
        "mean_face": mean_face,
        "scaler": (s_mean, s_var, s_scale),
        "pca": pca,
        "face_features": pca["fit_transform"],                # :143
        "eigenfaces": pca["components_"],                     # :137
    }


def sklearn_transform(p, scaler, pca):
    """``scaler.transform`` then ``pca.transform`` as in
    ``extract_face_features`` (scan-template-v4.py:265-266): sklearn
    ``_data.py:1096-1098`` and ``_base.py:148-155``."""
    s_mean, _, s_scale = scaler
    z = (np.asarray(p, dtype=np.float64) - s_mean) / s_scale
    comp = pca["components_"]
    return z @ comp.T - pca["mean_"] @ comp.T


def fold_projection(scaler, pca):
    """Fold StandardScaler + PCA.transform into one affine map
    ``f = (p - mu_f) . W`` with ``W = diag(1/sigma) . V^T`` and
    ``mu_f = mu + sigma * mu_pca``: the form the GPU projection consumes."""
    s_mean, _, s_scale = scaler
    w = (pca["components_"] / s_scale[None, :]).T
    mu_f = s_mean + s_scale * pca["mean_"]
    return mu_f, w


def project(p, mean, w):
    """``project_face_to_eigenspace`` batched (useless/scan.py:80-98):
    ``(p - mean) . W`` in float64."""
    return (np.asarray(p, dtype=np.float64) - np.asarray(mean, dtype=np.float64)) @ np.asarray(w, dtype=np.float64)


# --------------------------------------------------------------------------
# Recognise: similarity + arg-best (scan-template-v4.py:270-287, scan.py:58-132)
# --------------------------------------------------------------------------
def _unit_rows(a):
    a = np.asarray(a, dtype=np.float64)
    nrm = np.linalg.norm(a, axis=1, keepdims=True)
    out = np.zeros_like(a)
    nz = nrm[:, 0] > 0
    out[nz] = a[nz] / nrm[nz]
    return out


def cosine_scores(f, g):
    """``sklearn.metrics.pairwise.cosine_similarity(F, G)`` (pairwise.py:
    1730-1736): rows normalised, zero rows left at zero -> similarity 0
    (also the ``norm == 0`` branch of useless/scan.py:73-74)."""
    return _unit_rows(f) @ _unit_rows(g).T


def cosine_argmax(f, g):
    """First-max argmax of cosine similarity (scan-template-v4.py:274-276):
    returns ``(idx int64 (B,), best float64 (B,))``."""
    s = cosine_scores(f, g)
    idx = np.argmax(s, axis=1)
    return idx.astype(np.int64), s[np.arange(s.shape[0]), idx]


def l2_argmin(f, g, chunk=4096):
    """North-star L2 nearest neighbour: first-min argmin of squared
    Euclidean distance, computed in float64 in difference form so that the
    reported distance is accurate.  Returns ``(idx, dist2)``."""
    f = np.asarray(f, dtype=np.float64)
    g = np.asarray(g, dtype=np.float64)
    gn = (g * g).sum(axis=1)
    best_idx = np.empty(f.shape[0], dtype=np.int64)
    for s in range(0, f.shape[0], chunk):
        q = f[s:s + chunk]
        part = gn[None, :] - 2.0 * (q @ g.T)
        best_idx[s:s + chunk] = np.argmin(part, axis=1)
    diff = f - g[best_idx]
    return best_idx, (diff * diff).sum(axis=1)


def recognize_face_with_model(features, gallery, labels, person_id_map, threshold=0.7):
    """``recognize_face_with_model`` (scan-template-v4.py:270-287) for one
    probe: cosine vs every gallery row, first argmax, threshold with ``>=``,
    label via ``face_labels[idx]`` and the first matching name in
    ``person_id_map``; ``(-1, "unknown", sim)`` below threshold."""
    idx, best = cosine_argmax(np.asarray(features)[None, :], gallery)
    i, sim = int(idx[0]), float(best[0])
    if sim >= threshold:
        pid = labels[i]
        name = "unknown"
        for nm, v in person_id_map.items():
            if v == pid:
                name = nm
                break
        return pid, name, sim
    return -1, "unknown", sim


def recognize_face_manual(face_vector, model, threshold=0.7):
    """``recognize_face`` on a ``models/*_pca_model.pkl`` dict
    (useless/scan.py:100-132): project (:118), cosine against every
    ``projected_data`` row (:122-124), max (:127), ``>=`` threshold (:130)."""
    proj = project(np.asarray(face_vector)[None, :], model["mean_face"], model["eigenfaces"])
    s = cosine_scores(proj, model["projected_data"])[0]
    best = float(s.max())
    return model["person_name"], best, best >= threshold


# --------------------------------------------------------------------------
# Synthetic workload (SURVEY.md §8d generator), deterministic per seed.
# --------------------------------------------------------------------------
def synth_mean_face(side):
    """Smooth 128-centred face-like mean image, flattened (side*side,)."""
    yy, xx = np.mgrid[0:side, 0:side].astype(np.float64) / max(side - 1, 1)
    r2 = (xx - 0.5) ** 2 / 0.16 + (yy - 0.5) ** 2 / 0.25
    face = 128.0 + 50.0 * np.exp(-r2) - 25.0 * np.exp(-((xx - 0.33) ** 2 + (yy - 0.4) ** 2) / 0.004) \
        - 25.0 * np.exp(-((xx - 0.67) ** 2 + (yy - 0.4) ** 2) / 0.004)
    return face.ravel()


def synth_basis(d, r, seed=0):
    """Orthonormal (d, r) basis from the QR of a seeded Gaussian matrix."""
    rng = np.random.default_rng(seed)
    q, _ = np.linalg.qr(rng.standard_normal((d, r)))
    return q


def synth_spectrum(r):
    return 60.0 * (np.arange(r) + 1.0) ** -0.7


def synth_faces(n, side, r=64, seed=0, noise=2.0, basis=None, coeffs=None):
    """uint8 faces ``clip(round(mu0 + z.diag(s).B^T + eps))``.

    Returns ``(X uint8 (n, side*side), coeffs (n, r))``.
    """
    d = side * side
    rng = np.random.default_rng(seed + 1)
    b = synth_basis(d, r, seed) if basis is None else basis
    if coeffs is None:
        coeffs = rng.standard_normal((n, r)) * synth_spectrum(r)[None, :]
    x = synth_mean_face(side)[None, :] + coeffs @ b.T + noise * rng.standard_normal((n, d))
    return np.clip(np.rint(x), 0, 255).astype(np.uint8), coeffs


INT_SYNTH_BLOCK = 2048


def int_synth_spectrum(r):
    """Integer factor weights floor(4096 / sqrt(j+1)) (pure integer arithmetic)."""
    import math
    return np.array([math.isqrt(4096 * 4096 // (j + 1)) for j in range(r)], dtype=np.int64)


def light_like_spectrum(lam, r):
    """Integer factor weights whose covariance spectrum follows the eigenvalue profile
    ``lam`` of a real training set (tests/golden/light_stats.npz: the reference's
    faces/Light_version, useless/train.py:56-128) — its clustered eigen-gaps, the regime
    where eigenvector parity is hardest — then decays as 1/(j+1) past len(lam):
    ``s_j = round(4096 sqrt(lam_j / lam_0))`` (pure integer inputs for int_synth_faces)."""
    lam = np.asarray(lam, dtype=np.float64)
    w = np.empty(r)
    m = min(r, len(lam))
    w[:m] = np.sqrt(lam[:m] / lam[0])
    if r > m:
        w[m:] = w[m - 1] * np.sqrt(m / (np.arange(m, r) + 1.0))
    return np.maximum(1, np.rint(4096.0 * w)).astype(np.int64)


def int_synth_faces(n, side, r=160, seed=0, rows=None, spectrum=None):
    """Bit-reproducible synthetic faces for fit-parity fixtures at large shapes.

    ``X = clip(M + rint((Z.diag(s)).Bq / 2^20) + eps, 0, 255)`` with integer-valued
    operands only: ``Bq`` uniform integers in [-128, 128) (r x d), ``Z`` sums of four
    uniform integers in [-32, 32) per factor, ``s`` :func:`int_synth_spectrum`,
    ``eps`` uniform in {-2..2}, ``M`` an integer radial face-like mean.  Every partial
    sum of ``Z.diag(s).Bq`` is an integer below 2^53, so the float64 product is exact
    whatever BLAS kernel or summation order the host uses: the same seed gives the same
    pixels on the build container and on the GPU box.  Rows come in blocks of
    INT_SYNTH_BLOCK, each from its own seeded stream, so ``rows=(lo, hi)`` regenerates
    any slice.  The spectrum (eigenvalues ~ 1/(j+1) for r factors, noise floor far
    below) keeps the top-128 eigen-gaps meaningful for eigenvector parity; ``spectrum``
    (r integers in 0..4096) replaces it, e.g. :func:`light_like_spectrum`.
    """
    d = side * side
    lo, hi = (0, n) if rows is None else rows
    bq = np.random.default_rng([seed, 0]).integers(-128, 128, size=(r, d)).astype(np.float64)
    s = (int_synth_spectrum(r) if spectrum is None else np.asarray(spectrum, dtype=np.int64)).astype(np.float64)
    assert s.shape == (r,) and s.min() >= 0 and s.max() <= 4096, "integer weights 0..4096 keep the product exact"
    yy, xx = np.mgrid[0:side, 0:side]
    dy, dx = yy - side // 2, xx - side // 2
    m = (170 - (dx * dx + dy * dy) * 80 // max(side * side // 2, 1)).ravel().astype(np.float64)
    out = np.empty((hi - lo, d), dtype=np.uint8)
    for blk in range(lo // INT_SYNTH_BLOCK, (hi - 1) // INT_SYNTH_BLOCK + 1 if hi > lo else 0):
        a, e = blk * INT_SYNTH_BLOCK, min(n, (blk + 1) * INT_SYNTH_BLOCK)
        rng = np.random.default_rng([seed, 1, blk])
        z = rng.integers(-32, 32, size=(4, e - a, r)).sum(axis=0).astype(np.float64) * s
        eps = rng.integers(-2, 3, size=(e - a, d)).astype(np.float64)
        px = np.clip(m + np.rint((z @ bq) * (1.0 / 1048576.0)) + eps, 0, 255).astype(np.uint8)
        ca, ce = max(a, lo), min(e, hi)
        out[ca - lo:ce - lo] = px[ca - a:ce - a]
    return out


def planted_probes(gallery_pixels_fn, targets, noise=4.0, seed=7):
    """Probes = gallery faces + N(0, noise^2), re-quantised to uint8."""
    rng = np.random.default_rng(seed)
    base = gallery_pixels_fn(targets).astype(np.float64)
    return np.clip(np.rint(base + noise * rng.standard_normal(base.shape)), 0, 255).astype(np.uint8)


# --------------------------------------------------------------------------
# CPU baseline of record: the batched fp32 BLAS restatement of
# project (useless/scan.py:93-96) + L2 nearest neighbour, run on all host cores.
# --------------------------------------------------------------------------
def recognize_l2_f32(p, mean, w, g, gnorm2=None, chunk=65536):
    """``(p - mean) . W`` then ``argmin_j ||g_j||^2 - 2 f.g_j`` in float32 BLAS,
    gallery streamed in chunks.  Returns ``(idx, features)``."""
    f = (np.asarray(p, dtype=np.float32) - np.asarray(mean, dtype=np.float32)) @ np.asarray(w, dtype=np.float32)
    g = np.asarray(g, dtype=np.float32)
    if gnorm2 is None:
        gnorm2 = np.einsum("ij,ij->i", g, g)
    best = np.full(f.shape[0], np.inf, dtype=np.float32)
    idx = np.zeros(f.shape[0], dtype=np.int64)
    for s in range(0, g.shape[0], chunk):
        part = gnorm2[None, s:s + chunk] - 2.0 * (f @ g[s:s + chunk].T)
        j = np.argmin(part, axis=1)
        v = part[np.arange(part.shape[0]), j]
        upd = v < best
        best[upd] = v[upd]
        idx[upd] = j[upd] + s
    return idx, f
