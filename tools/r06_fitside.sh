#!/bin/bash
# Round 6: the covariance SYRK with C digit planes on the side stream (EF_FIT_SIDE=1, product) vs on the main stream (0)
# (product): C3 fit medians alternated, results compared (exact integers: identical), then
# a kernel trace of each.
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${1:-r06/fitside}
mkdir -p $O
export EF_LIB_VARIANT=diag
for v in 1 0 1b 0b; do
  EF_FIT_SIDE=${v:0:1} timeout -k 10 240 python tools/fit_ab.py $O/c3_$v.npz 5 > $O/c3_$v.txt 2>&1 || { echo "c3 rc=$?"; tail $O/c3_$v.txt; exit 1; }
  echo "side=$v $(grep median_s $O/c3_$v.txt)" >> $O/ab.txt
done
python - "$O" >> $O/ab.txt <<'PY'
import sys, numpy as np
o = sys.argv[1]
a, b = np.load(f"{o}/c3_1.npz"), np.load(f"{o}/c3_0.npz")
print("eigenvalues identical:", bool(np.array_equal(a["eigenvalues"], b["eigenvalues"])),
      "components identical:", bool(np.array_equal(a["components"], b["components"])))
PY
for v in 1 0; do
  EF_FIT_SIDE=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$v -o run -- python tools/fit_ab.py $O/x.npz 1 > $O/t_$v.txt 2>&1 || { echo "trace rc=$?"; tail $O/t_$v.txt; exit 1; }
  python - $O/trace_$v/run_kernel_stats.csv $v >> $O/ab.txt <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'oz_rows' in r['Name'] or 'syrk16_i8_kernel<6' in r['Name']: print('side', sys.argv[2], r['Name'][:60], r['Calls'], float(r['AverageNs']) / 1e6, 'ms')
PY
done
cat $O/ab.txt
