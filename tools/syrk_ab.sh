#!/bin/bash
# SYRK tile A/B: fit parity tests on the product library, then the C3 fit timed with the
# diagnostic build at 256 x 256 and 256 x 384 tiles, and a kernel trace of the product fit.
# usage: bash tools/syrk_ab.sh <tag>
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_fit.py -x -q --timeout 300 -p no:cacheprovider > $O/pytest.txt 2>&1
rc=$?
tail -3 $O/pytest.txt
[ $rc -ne 0 ] && exit $rc
for tj in 256 384 256 384; do
  EF_LIB_VARIANT=diag EF_SYRK_TJ=$tj timeout -k 10 200 python tools/prof_fit.py > $O/fit_tj$tj.txt 2>&1 || exit $?
  echo "tj=$tj $(grep -o "'gpu_fit_s': [0-9.]*" $O/fit_tj$tj.txt)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/fr -o run -- python tools/prof_fit.py > $O/out.txt 2>&1 || exit $?
python tools/fit_breakdown.py /tmp/fr/run_kernel_trace.csv > $O/breakdown.txt && cp /tmp/fr/run_kernel_stats.csv $O/kernel_stats.csv
head -4 $O/breakdown.txt
