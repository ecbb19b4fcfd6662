#!/bin/bash
# Round 6: block-Jacobi pair solves with every thread computing its own two rotations (one
# barrier per inner round; product lib) vs the published rotations (libeigenface_old.so, a
# copy of the previous product build): C3 fit medians alternated, results compared, kernel
# traces, then the fit / eigensolver GPU tests on the new build.
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${1:-r06/bjrot}
mkdir -p $O
for v in new old new2 old2; do
  case $v in old*) export EF_LIB_VARIANT=old;; *) unset EF_LIB_VARIANT;; esac
  timeout -k 10 240 python tools/fit_ab.py $O/c3_$v.npz 5 > $O/c3_$v.txt 2>&1 || { echo "c3 rc=$?"; tail $O/c3_$v.txt; exit 1; }
  echo "$v $(grep median_s $O/c3_$v.txt)" >> $O/ab.txt
done
python - "$O" >> $O/ab.txt <<'PY'
import sys, numpy as np
o = sys.argv[1]
a, b = np.load(f"{o}/c3_new.npz"), np.load(f"{o}/c3_old.npz")
ev = np.abs(a["eigenvalues"] - b["eigenvalues"]) / np.abs(b["eigenvalues"])
ca, cb = a["components"], b["components"]
s = np.sign(np.sum(ca * cb, axis=1, keepdims=True))
print(f"eigenvalues max rel diff {ev.max():.3e}; components max abs diff {np.abs(ca * s - cb).max():.3e}")
PY
rm -f $O/*.npz
for v in new old; do
  case $v in old*) export EF_LIB_VARIANT=old;; *) unset EF_LIB_VARIANT;; esac
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$v -o run -- python tools/fit_ab.py $O/x.npz 1 > $O/t_$v.txt 2>&1 || { echo "trace rc=$?"; tail $O/t_$v.txt; exit 1; }
  python - $O/trace_$v/run_kernel_stats.csv $v >> $O/ab.txt <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'bj_round' in r['Name']: print(sys.argv[2], r['Name'][:40], r['Calls'], float(r['TotalDurationNs']) / 1e6, 'ms total', float(r['AverageNs']) / 1e3, 'us avg')
PY
done
rm -f $O/*.npz
cat $O/ab.txt
unset EF_LIB_VARIANT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_manual.py tests/test_gpu_fit.py tests/test_gpu_sharded_fit.py tests/test_gpu_c2_full.py tests/test_gpu_compat.py tests/test_gpu_dropin.py > $O/pytest.txt 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
