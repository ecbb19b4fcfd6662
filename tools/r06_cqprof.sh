#!/bin/bash
# kernel trace of the C3 fit with the int8-digit C.Q products (diagnostic build)
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${1:-r06/cqprof}
mkdir -p $O
export EF_LIB_VARIANT=diag EF_FIT_CQ_I8=${2:-1}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python tools/fit_ab.py $O/x.npz 1 > $O/run.txt 2>&1 || { echo "rc=$?"; tail $O/run.txt; exit 1; }
head -25 $O/trace/run_kernel_stats.csv | cut -d, -f1-5
