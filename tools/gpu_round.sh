#!/bin/bash
# One GPU session: parity tests, bench, rocprof kernel trace + PMC passes.
# usage: bash tools/gpu_round.sh <tag>     (outputs under gpurun_out/<tag>/)
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
TAG=${1:-run}
O=gpurun_out/$TAG
mkdir -p $O
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  echo "== $name: $*" >> $O/steps.log
  timeout -k 10 $to "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "== $name rc=$rc" >> $O/steps.log
  return $rc
}
step pytest 600 python -m pytest tests -m gpu -q --timeout 300 -p no:cacheprovider; rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
step bench 600 python bench.py || exit $?
[ "$2" = quick ] && { echo done >> $O/steps.log; exit 0; }
B="bench.py --steps 5 --warmup 2 --no-cpu --no-fit --no-c2 --no-c5 --no-image"
step trace 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python $B || exit $?
step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python $B || exit $?
step pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python $B || exit $?
step pmc_sq 600 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY --output-format csv -d $O/pmc_sq -o run -- python $B || exit $?
echo done >> $O/steps.log
