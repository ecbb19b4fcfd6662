#!/bin/bash
# Round 6: the fit's fine-phase products C.Q on the int8 matrix cores (Ozaki-style digit
# pairs) against the fp64 MFMA product: C3 fit with EF_FIT_CQ_I8=1 / 0 (diagnostic build;
# iterations, time, residual trace, eigenvalue / component differences), then the fit tests.
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${1:-r06/cq}
mkdir -p $O
export EF_FIT_DEBUG=1
for v in 1 0; do
  EF_LIB_VARIANT=diag EF_FIT_CQ_I8=$v timeout -k 10 240 python tools/fit_ab.py $O/c3_$v.npz 5 > $O/c3_$v.txt 2>&1 || { echo "c3 rc=$?"; tail $O/c3_$v.txt; exit 1; }
  echo "C3 cq_i8=$v: $(grep 'rr it' $O/c3_$v.txt | tail -4 | tr '\n' ' ') $(grep median_s $O/c3_$v.txt)" >> $O/ab.txt
done
python - "$O" >> $O/ab.txt <<'PY'
import sys, numpy as np
o = sys.argv[1]
a, b = np.load(f"{o}/c3_1.npz"), np.load(f"{o}/c3_0.npz")
ev = np.abs(a["eigenvalues"] - b["eigenvalues"]) / np.abs(b["eigenvalues"])
ca, cb = a["components"], b["components"]
s = np.sign(np.sum(ca * cb, axis=1, keepdims=True))
print(f"eigenvalues max rel diff {ev.max():.3e}; components max abs diff {np.abs(ca * s - cb).max():.3e}")
PY
cat $O/ab.txt
unset EF_FIT_DEBUG
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_manual.py tests/test_gpu_fit.py > $O/pytest.txt 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
