#!/bin/bash
# Round 6: placement of the Rayleigh-Ritz step after a gap-rule miss — rho^p >= 1.5 need
# (product default) against the first form T_p >= 2 need (EF_FIT_GAP_MARGIN=0), C3 fit
# (diagnostic build), then the fit tests on the product build.
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${1:-r06/gapsched}
mkdir -p $O
export EF_FIT_DEBUG=1
for v in 1.5 0; do
  EF_LIB_VARIANT=diag EF_FIT_GAP_MARGIN=$v timeout -k 10 240 python tools/fit_ab.py $O/c3_$v.npz 5 > $O/c3_$v.txt 2>&1 || { echo "c3 rc=$?"; tail $O/c3_$v.txt; exit 1; }
  echo "C3 gap margin $v: $(grep 'rr it' $O/c3_$v.txt | tail -4 | tr '\n' ' ') $(grep median_s $O/c3_$v.txt)" >> $O/ab.txt
done
python - "$O" >> $O/ab.txt <<'PY'
import sys, numpy as np
o = sys.argv[1]
a, b = np.load(f"{o}/c3_1.5.npz"), np.load(f"{o}/c3_0.npz")
ev = np.abs(a["eigenvalues"] - b["eigenvalues"]) / np.abs(b["eigenvalues"])
ca, cb = a["components"], b["components"]
s = np.sign(np.sum(ca * cb, axis=1, keepdims=True))
print(f"eigenvalues max rel diff {ev.max():.3e}; components max abs diff {np.abs(ca * s - cb).max():.3e}")
PY
cat $O/ab.txt
unset EF_FIT_DEBUG
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_manual.py tests/test_gpu_fit.py -s > $O/pytest.txt 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.txt; exit 1; }
grep -E "dark:|C3 1M|r/gap" $O/pytest.txt | head; tail -1 $O/pytest.txt
