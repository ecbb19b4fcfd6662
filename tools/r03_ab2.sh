#!/bin/bash
# Second A/B session: JPEG/Haar tests, SYRK 32x32x32 vs 16x16x64 (B-fragment ring), streamed JPEG ingest.  usage: bash tools/r03_ab2.sh <tag>
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_jpeg.py -x -q --timeout 300 -p no:cacheprovider > $O/pytest.txt 2>&1 || exit $?
EF_LIB_VARIANT=diag timeout -k 10 400 python -u tools/syrk16_check.py > $O/syrk16.txt 2>&1 || exit $?
timeout -k 10 200 python -u tools/jpeg_async_prof.py > $O/jpeg_async.txt 2>&1 || exit $?
