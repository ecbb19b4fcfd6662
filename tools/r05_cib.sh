#!/bin/bash
# CholQR microbenchmark (tools/micro/chol_inv_bench.cpp), its kernel split, phase stamps.
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${1:-r05/cib}
mkdir -p $O
timeout -k 10 60 tools/micro/bin/cib 256 128 88 200 > $O/cib.txt 2>&1 || { echo "cib rc=$?"; cat $O/cib.txt; exit 1; }
cat $O/cib.txt
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/cibprof -o run -- tools/micro/bin/cib 256 > $O/cibprof.txt 2>&1 || { echo "cibprof rc=$?"; exit 1; }
timeout -k 10 60 tools/micro/bin/cib_stamp 256 > $O/cib_stamp.txt 2>&1 || { echo "stamp rc=$?"; exit 1; }
cat $O/cib_stamp.txt
