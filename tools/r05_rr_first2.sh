#!/bin/bash
# First Rayleigh-Ritz tolerance: the fit GPU tests with the new default, and C2-shape
# fits (Gram path, early Rayleigh-Ritz steps) timed against the old value.
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${1:-r05/rrfirst2}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_fit.py tests/test_gpu_manual.py tests/test_gpu_sharded_fit.py > $O/pytest.txt 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
export EF_LIB_VARIANT=diag EF_FIT_DEBUG=1
for t in 1e-4 1e-2; do
  EF_FIT_RR_FIRST=$t timeout -k 10 300 python - > $O/c2_$t.txt 2>&1 <<'PY' || { echo "c2 rc=$?"; exit 1; }
import sys, time, os
sys.path.insert(0, "face-detection-recognization-pca_amd"); sys.path.insert(0, ".")
import numpy as np, torch
from oracle import eigenface_oracle as orc
from eigenface import Engine
eng = Engine(0)
for n in (2000, 10000):
    x, _ = orc.synth_faces(n, 128, r=256, seed=n)
    xd = torch.from_numpy(x).cuda()
    eng.fit(xd, 64, projection=False)
    ts = []
    for _ in range(5):
        torch.cuda.synchronize(); t = time.perf_counter()
        r = eng.fit(xd, 64, projection=False)
        torch.cuda.synchronize(); ts.append(time.perf_counter() - t)
    print("n", n, "median_s", round(float(np.median(ts)), 4), "iters", r.iters, "lam0", float(r.eigenvalues[0]), flush=True)
PY
  grep -E "median_s|sweeps=" $O/c2_$t.txt | sed "s/^/tol $t: /" >> $O/ab.txt
done
cat $O/ab.txt
