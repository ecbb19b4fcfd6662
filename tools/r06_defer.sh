#!/bin/bash
# Round 6: the fit with the CholQR check deferred to the Rayleigh-Ritz steps (EF_FIT_DEFER=1, product) vs every iteration (0)
# (product): C3 fit medians alternated, results compared (exact integers: identical), then
# a kernel trace of each.
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${1:-r06/defer}
mkdir -p $O
export EF_LIB_VARIANT=diag EF_FIT_DEBUG=1
for v in 1 0 1b 0b; do
  EF_FIT_DEFER=${v:0:1} timeout -k 10 240 python tools/fit_ab.py $O/c3_$v.npz 5 > $O/c3_$v.txt 2>&1 || { echo "c3 rc=$?"; tail $O/c3_$v.txt; exit 1; }
  echo "defer=$v $(grep 'rr it' $O/c3_$v.txt | tail -2 | tr '\n' ' ') $(grep median_s $O/c3_$v.txt)" >> $O/ab.txt
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
for v in 1 0; do
  EF_FIT_DEFER=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$v -o run -- python tools/fit_ab.py $O/x.npz 1 > $O/t_$v.txt 2>&1 || { echo "trace rc=$?"; tail $O/t_$v.txt; exit 1; }
  python - $O/trace_$v/run_kernel_stats.csv $v >> $O/ab.txt <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'chol_blk' in r['Name']: print('defer', sys.argv[2], r['Name'][:60], r['Calls'], float(r['AverageNs']) / 1e6, 'ms')
PY
done
cat $O/ab.txt
unset EF_LIB_VARIANT EF_FIT_DEBUG
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_manual.py tests/test_gpu_fit.py tests/test_gpu_sharded_fit.py tests/test_gpu_c2_full.py > $O/pytest.txt 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.txt; exit 1; }
grep -E "retries_checked|PASS.*1M" $O/pytest.txt || true; tail -1 $O/pytest.txt
