#!/bin/bash
# Template localiser on template sets whose pieces need <= 5 k-blocks: the 71 KiB
# (two workgroups per CU) corr kernel vs the 148 KiB one.  usage: bash tools/tm_narrow_ab.sh <tag>
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/$1
mkdir -p $O
EF_LIB_VARIANT=diag timeout -k 10 200 python -u tools/tm_micro.py > $O/micro_narrow.txt 2>&1 || exit $?
EF_LIB_VARIANT=diag EF_TM_WIDE=1 timeout -k 10 200 python -u tools/tm_micro.py > $O/micro_wide.txt 2>&1 || exit $?
EF_LIB_VARIANT=diag timeout -k 10 200 python -u tools/tm_micro.py > $O/micro_narrow2.txt 2>&1 || exit $?
