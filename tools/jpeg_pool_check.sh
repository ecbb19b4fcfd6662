#!/bin/bash
# JPEG tests + streamed ingest profile + host stages (diagnostic build) after moving the
# host parse / destuff onto the persistent pool.  usage: bash tools/jpeg_pool_check.sh <tag>
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/$1
mkdir -p $O
nproc > $O/nproc.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_jpeg.py tests/test_gpu_compat.py -x -q --timeout 300 -p no:cacheprovider > $O/pytest.txt 2>&1 || exit $?
timeout -k 10 200 python -u tools/jpeg_async_prof.py > $O/async.txt 2>&1 || exit $?
EF_LIB_VARIANT=diag EF_JPEG_TIMES=1 timeout -k 10 200 python -u tools/jpeg_async_prof.py > $O/stages.txt 2>&1 || exit $?
