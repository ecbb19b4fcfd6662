#!/bin/bash
# Round 6: the training projection on 256 x 384 tiles (product: 6 digits x kk = 128 = 2
# tiles) vs 256 x 256 (libeigenface_old.so, a copy of the previous product build): the
# bench C3 fit + transform legs alternated, a kernel trace of each, then the fit / drop-in
# GPU tests on the new build.
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${1:-r06/proj384}
mkdir -p $O
for v in new old new2 old2; do
  case $v in old*) export EF_LIB_VARIANT=old;; *) unset EF_LIB_VARIANT;; esac
  timeout -k 10 400 python bench.py --steps 2 --warmup 1 --repeats 1 --no-cpu --no-c2 --no-c5 --no-image > $O/b_$v.json 2> $O/b_$v.err || { echo "bench rc=$?"; tail $O/b_$v.err; exit 1; }
  python - $O/b_$v.json $v >> $O/ab.txt <<'PY'
import json, sys
f = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])["fit"]["c3"]
print(sys.argv[2], "fit", f["gpu_fit_s"], "fit+transform", f["gpu_fit_transform_s"], f["gpu_fit_transform_s_repeats"], "iters", f["eigensolver_iters"])
PY
done
for v in new old; do
  case $v in old*) export EF_LIB_VARIANT=old;; *) unset EF_LIB_VARIANT;; esac
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$v -o run -- python tools/prof_fit.py > $O/t_$v.txt 2>&1 || { echo "trace rc=$?"; tail $O/t_$v.txt; exit 1; }
  python - $O/trace_$v/run_kernel_stats.csv $v >> $O/ab.txt <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'proj_i8' in r['Name'] or 'proj_combine' in r['Name']: print(sys.argv[2], r['Name'][:50], r['Calls'], float(r['AverageNs']) / 1e6, 'ms avg')
PY
done
cat $O/ab.txt
unset EF_LIB_VARIANT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fit.py tests/test_gpu_manual.py tests/test_gpu_dropin.py tests/test_gpu_compat.py tests/test_gpu_sharded_fit.py > $O/pytest.txt 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
