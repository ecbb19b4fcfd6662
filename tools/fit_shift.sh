#!/bin/bash
# Spectral-shift A/B: fit parity tests (product library), then C3 + C2 fits with the
# diagnostic library, shift off / on.  usage: bash tools/fit_shift.sh <tag>
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_fit.py tests/test_gpu_dropin.py -x -q --timeout 300 -p no:cacheprovider > $O/pytest.txt 2>&1
rc=$?
tail -3 $O/pytest.txt
[ $rc -ne 0 ] && exit $rc
for sh in 0 1; do
  EF_LIB_VARIANT=diag EF_FIT_SHIFT=$sh EF_FIT_DEBUG=1 timeout -k 10 300 python tools/prof_fit2.py > $O/shift$sh.txt 2> $O/shift$sh.err || exit $?
  echo "shift=$sh $(tail -1 $O/shift$sh.txt)"
done
