#!/bin/bash
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/r06/bench1
mkdir -p $O
timeout -k 10 900 python bench.py > $O/bench.txt 2> $O/bench.err || { echo "bench rc=$?"; tail -20 $O/bench.err; exit 1; }
tail -c 3000 $O/bench.txt
bash tools/jpeg_host_stages.sh r06/jpegstages
