#!/bin/bash
# rocprofv3 kernel trace of the C3 fit (tools/prof_fit.py) + per-kernel breakdown of the
# last fit.  usage: bash tools/fit_prof.sh <tag>   (outputs under gpurun_out/<tag>/)
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/fr -o run -- python tools/prof_fit.py > $O/out.txt 2>&1 || exit $?
python tools/fit_breakdown.py /tmp/fr/run_kernel_trace.csv > $O/breakdown.txt && cp /tmp/fr/run_kernel_stats.csv $O/kernel_stats.csv
cat $O/breakdown.txt
