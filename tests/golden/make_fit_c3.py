"""Fit-parity fixture at the C3 fit shape (d = 128 x 128 = 16384, k = 128, n >= d).

The GPU fit at this shape takes the covariance branch (order 16384), the order >= 12288
Rayleigh-Ritz schedule and the fp32 coarse phase of the subspace iteration — paths no
small fixture reaches.  This script runs the CPU oracle's covariance-branch restatement
(:func:`oracle.eigenface_oracle.pca_cov_fit`, useless/train.py:97-103 with the
StandardScaler of train-v4.py:131) on ``int_synth_faces(20000, 128, r=160, seed=0)`` —
an exact-integer generator, so the GPU test regenerates the identical pixels on the box
— and commits a compact summary:

* ``eigenvalues`` (128), ``total_var``;
* ``comps_R`` = components_ @ R for a fixed Rademacher R (16384 x 8, seed 5): every
  pixel of every component enters the check;
* ``comps_px`` = components_ at 256 fixed pixel positions;
* ``features`` = fit_transform rows 0..63;
* ``scaler_mean`` / ``scaler_scale``;
* ``top_idx`` / ``top_val`` (k x 2): per component, the pixels of its two largest |entries|
  and their (svd_flip-signed) values — the sklearn sign rule (extmath.py:946-952) keys on
  the first, so a component whose two are nearly tied may legitimately come out with the
  other sign from a fit whose rounding differs; the GPU test allows a flip only there.

The oracle itself is pinned against the reference's own outputs at smaller shapes
(tests/golden/make_goldens.py, tests/test_oracle_golden.py), and pca_cov_fit against
pca_full_fit (the SVD restatement) in tests/test_oracle_golden.py.

Usage:  python tests/golden/make_fit_c3.py     (~10 min on 8 cores, ~12 GB RAM)
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.abspath(os.path.join(HERE, "..", "..")))
from oracle import eigenface_oracle as orc  # noqa: E402

N, SIDE, R_FACT, SEED, K = 20000, 128, 160, 0, 128


def probe_matrices(d):
    r = np.random.default_rng([5]).integers(0, 2, size=(d, 8)).astype(np.float64) * 2.0 - 1.0
    px = np.sort(np.random.default_rng([6]).choice(d, size=256, replace=False))
    return r, px


def main():
    t0 = time.time()
    X = orc.int_synth_faces(N, SIDE, r=R_FACT, seed=SEED)
    print(f"generated {X.shape} in {time.time() - t0:.1f} s")
    t0 = time.time()
    res = orc.pca_cov_fit(X, K, standardize=True)
    print(f"oracle fit in {time.time() - t0:.1f} s")
    R, px = probe_matrices(X.shape[1])
    comps = res["components_"]
    top_idx = np.argsort(-np.abs(comps), axis=1, kind="stable")[:, :2]
    np.savez_compressed(
        os.path.join(HERE, "fit_c3.npz"),
        n=N, side=SIDE, r=R_FACT, seed=SEED, k=K,
        eigenvalues=res["explained_variance_"], total_var=res["total_var"],
        comps_R=comps @ R, comps_px=comps[:, px], px=px,
        features=res["fit_transform"][:64],
        scaler_mean=res["scaler"][0], scaler_scale=res["scaler"][2],
        top_idx=top_idx, top_val=np.take_along_axis(comps, top_idx, axis=1),
    )
    lam = res["explained_variance_"]
    print("top eigenvalues", lam[:4], "lambda_128", lam[-1], "min rel gap",
          float(np.min(-np.diff(lam) / lam[1:])))


if __name__ == "__main__":
    main()
