#!/bin/bash
# Round-3 A/B session on one box: int8 MFMA clock ceiling, SYRK 32x32x32 vs 16x16x64 (identity
# + C3 fit time), streamed JPEG ingest breakdown, and
# the covariance operand copy A/B.  usage: bash tools/r03_ab.sh <tag>
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_jpeg.py tests/test_gpu_haar.py -x -q --timeout 300 -p no:cacheprovider > $O/pytest.txt 2>&1 || exit $?
timeout -k 10 120 ./tools/micro/bf16_clock i > $O/i8_clock.json 2> $O/i8_clock.err || exit $?
EF_LIB_VARIANT=diag timeout -k 10 400 python -u tools/syrk16_check.py > $O/syrk16.txt 2>&1 || exit $?
timeout -k 10 200 python -u tools/jpeg_async_prof.py > $O/jpeg_async.txt 2>&1 || exit $?
bash tools/transpose_ab.sh $1_tab || exit $?
