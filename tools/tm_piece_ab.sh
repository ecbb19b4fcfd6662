#!/bin/bash
# Template localiser: 352-column pieces (one 148 KiB workgroup per CU) vs narrow pieces
# (MAXNKB <= 5: 71 KiB, two workgroups per CU) — parity under each width (diagnostic build,
# EF_TM_PIECE) and the bench's localiser line.  usage: bash tools/tm_piece_ab.sh <tag>
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_image.py -x -q --timeout 120 -p no:cacheprovider > $O/pytest.txt 2>&1 || exit $?
for P in 128 96; do
  EF_LIB_VARIANT=diag EF_TM_PIECE=$P timeout -k 10 300 python -u -m pytest tests/test_gpu_image.py -x -q --timeout 120 -p no:cacheprovider -k "template or localiser" > $O/pytest_p$P.txt 2>&1 || exit $?
done
for P in 352 128 96 64; do
  EF_LIB_VARIANT=diag EF_TM_PIECE=$P timeout -k 10 200 python -u tools/prof_image.py > $O/img_p$P.json 2>&1 || exit $?
done
EF_LIB_VARIANT=diag EF_TM_PIECE=128 timeout -k 10 200 python -u tools/tm_micro.py > $O/micro_p128.txt 2>&1 || exit $?
timeout -k 10 200 python -u tools/tm_micro.py > $O/micro_p352.txt 2>&1 || exit $?
