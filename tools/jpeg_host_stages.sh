#!/bin/bash
# Host stages of the streamed JPEG ingest (diagnostic build, EF_JPEG_TIMES: parse, pinned,
# destuff, tables per call; the device stages synchronise, so the wall here is not the
# streamed one).  usage: bash tools/jpeg_host_stages.sh <tag>
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/$1
mkdir -p $O
nproc > $O/nproc.txt
timeout -k 10 200 python -u tools/jpeg_async_prof.py > $O/async.txt 2>&1 || exit $?
EF_LIB_VARIANT=diag EF_JPEG_TIMES=1 timeout -k 10 200 python -u tools/jpeg_async_prof.py > $O/stages.txt 2>&1 || exit $?
