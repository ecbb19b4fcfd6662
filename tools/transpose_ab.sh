#!/bin/bash
# A/B of the covariance operand copy (transpose_stats_kernel vs transpose_stats_lds_kernel)
# inside the C3 fit: two kernel traces of tools/prof_fit.py with the diagnostic build,
# EF_TRANSPOSE_LDS=0 / 1, then each trace's transpose kernel line.  usage: bash tools/transpose_ab.sh <tag>
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/$1
mkdir -p $O
for v in 0 1 0 1; do
  EF_LIB_VARIANT=diag EF_TRANSPOSE_LDS=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d /tmp/ta$v -o run -- python tools/prof_fit.py > $O/fit_$v.txt 2>&1 || exit $?
  grep -E "transpose_stats|syrk_i8" /tmp/ta$v/run_kernel_stats.csv >> $O/ab_$v.txt
  tail -1 $O/fit_$v.txt >> $O/ab_$v.txt
done
