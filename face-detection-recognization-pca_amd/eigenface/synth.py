"""Deterministic synthetic eigenfaces workload (SURVEY.md §8d generator).

Faces are ``clip(round(mu0 + z . diag(s) . B^T + eps))`` with a smooth face-like mean
``mu0``, an orthonormal basis ``B`` (d x k), spectrum ``s_j = 60 (j+1)^-0.7`` and
per-pixel noise.  Gallery features are the coefficients ``z . diag(s)`` (what the
projection of a noise-free gallery face onto ``B`` returns); probes are gallery faces
rendered to pixels with noise, so every probe has a known nearest neighbour.

Rows are generated in fixed blocks from per-block seeds, so any rank can regenerate
exactly the rows it owns and the probes' targets.
"""
from __future__ import annotations

import numpy as np

BLOCK = 65536


def mean_face(side: int) -> np.ndarray:
    yy, xx = np.mgrid[0:side, 0:side].astype(np.float64) / max(side - 1, 1)
    r2 = (xx - 0.5) ** 2 / 0.16 + (yy - 0.5) ** 2 / 0.25
    face = 128.0 + 50.0 * np.exp(-r2) - 25.0 * np.exp(-((xx - 0.33) ** 2 + (yy - 0.4) ** 2) / 0.004) \
        - 25.0 * np.exp(-((xx - 0.67) ** 2 + (yy - 0.4) ** 2) / 0.004)
    return face.ravel()


def spectrum(k: int) -> np.ndarray:
    return 60.0 * (np.arange(k) + 1.0) ** -0.7


def basis(d: int, k: int, seed: int = 0) -> np.ndarray:
    """Orthonormal d x k basis (QR of a seeded Gaussian), float64."""
    rng = np.random.default_rng(seed)
    q, _ = np.linalg.qr(rng.standard_normal((d, k)))
    return q


def gallery_rows(lo: int, hi: int, k: int, seed: int = 1) -> np.ndarray:
    """Gallery feature rows [lo, hi) as float32 (n x k)."""
    s = spectrum(k).astype(np.float32)
    out = np.empty((hi - lo, k), dtype=np.float32)
    b0 = lo // BLOCK
    b1 = (hi - 1) // BLOCK if hi > lo else b0 - 1
    for blk in range(b0, b1 + 1):
        rng = np.random.default_rng((seed, blk))
        z = rng.standard_normal((BLOCK, k), dtype=np.float32) * s
        a = max(lo, blk * BLOCK)
        e = min(hi, (blk + 1) * BLOCK)
        out[a - lo:e - lo] = z[a - blk * BLOCK:e - blk * BLOCK]
    return out


def probes(targets: np.ndarray, n_gallery: int, k: int, side: int, noise: float = 2.0,
           seed: int = 1, basis_seed: int = 0, B: np.ndarray | None = None) -> np.ndarray:
    """uint8 probe faces (len(targets) x side*side) rendered from gallery rows."""
    d = side * side
    B = basis(d, k, basis_seed) if B is None else B
    feats = np.empty((len(targets), k), dtype=np.float32)
    for blk in np.unique(targets // BLOCK):
        rows = gallery_rows(blk * BLOCK, min((blk + 1) * BLOCK, n_gallery), k, seed)
        sel = targets // BLOCK == blk
        feats[sel] = rows[targets[sel] - blk * BLOCK]
    rng = np.random.default_rng(seed + 12345)
    pix = mean_face(side)[None, :] + feats.astype(np.float64) @ B.T
    pix += noise * rng.standard_normal(pix.shape)
    return np.clip(np.rint(pix), 0, 255).astype(np.uint8)
