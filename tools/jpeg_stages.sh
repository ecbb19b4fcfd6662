#!/bin/bash
# JPEG ingest host/device stage times on the box (diagnostic library's stage timer).
# usage: bash tools/jpeg_stages.sh <tag>
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/$1
mkdir -p $O
EF_LIB_VARIANT=diag EF_JPEG_TIMES=1 timeout -k 10 300 python tools/micro/jpeg_prof.py > $O/prof.txt 2> $O/stages.txt || exit $?
timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu --no-fit --no-image --repeats 2 > $O/c5.out 2> $O/c5.err || exit $?
echo done
