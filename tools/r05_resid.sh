#!/bin/bash
# Ritz-residual acceptance study (diagnostic build): residuals at every fp64 Rayleigh-Ritz
# step (EF_FIT_DEBUG) on the C3 fit and C2 / C3-shape fits, then EF_FIT_RESID_TOL values
# against the value-change test alone: iterations, time, and the eigenvalue / component
# differences from the default fit.
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${1:-r05/resid}
mkdir -p $O
export EF_LIB_VARIANT=diag EF_FIT_DEBUG=1 O
for t in 0 1e-11 1e-10 1e-9; do
  EF_FIT_RESID_TOL=$t timeout -k 10 240 python tools/fit_ab.py $O/c3_$t.npz 5 > $O/c3_$t.txt 2>&1 || { echo "c3 rc=$?"; tail $O/c3_$t.txt; exit 1; }
  echo "C3 tol $t: $(grep 'rr it' $O/c3_$t.txt | tail -4 | tr '\n' ' ') $(grep median_s $O/c3_$t.txt)" >> $O/ab.txt
  EF_FIT_RESID_TOL=$t timeout -k 10 300 python - > $O/small_$t.txt 2>&1 <<'PY' || { echo "small rc=$?"; tail $O/small_$t.txt; exit 1; }
import sys, time, os
sys.path.insert(0, "face-detection-recognization-pca_amd"); sys.path.insert(0, ".")
import numpy as np, torch
from oracle import eigenface_oracle as orc
from eigenface import Engine
eng = Engine(0)
tag = os.environ["EF_FIT_RESID_TOL"]
for n, side, k, std in ((2000, 128, 64, False), (10000, 128, 64, False), (20000, 128, 128, True)):
    x, _ = orc.synth_faces(n, side, r=256, seed=n)
    xd = torch.from_numpy(x).cuda()
    eng.fit(xd, k, standardize=std, projection=False)
    ts = []
    for _ in range(3):
        torch.cuda.synchronize(); t = time.perf_counter()
        r = eng.fit(xd, k, standardize=std, projection=False)
        torch.cuda.synchronize(); ts.append(time.perf_counter() - t)
    np.savez(f"{os.environ['O']}/small_{tag}_{n}.npz", ev=r.eigenvalues.cpu().numpy(), comps=r.components.cpu().numpy())
    print("n", n, "median_s", round(float(np.median(ts)), 4), "iters", r.iters, flush=True)
PY
  grep -E "median_s" $O/small_$t.txt | sed "s/^/small tol $t: /" >> $O/ab.txt
done
python - >> $O/ab.txt <<PY
import numpy as np
def cmp(a, b):
    ea, eb = a["ev"] if "ev" in a.files else a["eigenvalues"], b["ev"] if "ev" in b.files else b["eigenvalues"]
    ca, cb = a["comps"] if "comps" in a.files else a["components"], b["comps"] if "comps" in b.files else b["components"]
    s = np.sign((ca * cb).sum(axis=1))
    return float(np.max(np.abs(ea - eb) / np.abs(ea))), float(np.max(np.abs(ca - cb * s[:, None])))
for t in ("1e-11", "1e-10", "1e-9"):
    print("C3", t, "vs 0: eig rel, comp abs", cmp(np.load("$O/c3_0.npz"), np.load(f"$O/c3_{t}.npz")))
    for n in (2000, 10000, 20000):
        print("small", n, t, "vs 0:", cmp(np.load(f"$O/small_0_{n}.npz"), np.load(f"$O/small_{t}_{n}.npz")))
PY
cat $O/ab.txt
