#!/bin/bash
# Fit check: fit parity tests, the C3 fit timed twice on the product library, the per-kernel
# breakdown of one fit under rocprofv3, then the diagnostic fp32-switch sweep (fit_tol.sh).
# usage: bash tools/fit_check.sh <tag> [sweep]
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_fit.py -x -q --timeout 300 -p no:cacheprovider > $O/pytest.txt 2>&1
rc=$?
tail -3 $O/pytest.txt
[ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  timeout -k 10 200 python tools/prof_fit.py > $O/fit_$r.txt 2>&1 || exit $?
  echo "fit $(grep -o "'gpu_fit_s': [0-9.]*" $O/fit_$r.txt) $(grep -o "'eigensolver_iters': [0-9]*" $O/fit_$r.txt)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/fr -o run -- python tools/prof_fit.py > $O/out.txt 2>&1 || exit $?
python tools/fit_breakdown.py /tmp/fr/run_kernel_trace.csv > $O/breakdown.txt && cp /tmp/fr/run_kernel_stats.csv $O/kernel_stats.csv
head -12 $O/breakdown.txt
[ "$2" = sweep ] && bash tools/fit_tol.sh $1_tol
exit 0
