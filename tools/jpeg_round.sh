#!/bin/bash
# JPEG session: GPU JPEG tests, streamed ingest breakdown, single-call chunk-size sweep.
# usage: bash tools/jpeg_round.sh <tag>
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_jpeg.py -x -q --timeout 300 -p no:cacheprovider > $O/pytest.txt 2>&1 || exit $?
timeout -k 10 200 python -u tools/jpeg_async_prof.py > $O/jpeg_async.txt 2>&1 || exit $?
timeout -k 10 300 python -u tools/micro/jpeg_prof.py 0 2048 3072 8192 > $O/jpeg_chunks.txt 2>&1 || exit $?
