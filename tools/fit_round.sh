#!/bin/bash
# GPU fit check: fit parity tests, then a rocprofv3 kernel trace of the C3 fit with the
# per-kernel breakdown of the last fit.  usage: bash tools/fit_round.sh <tag>
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_fit.py -x -q --timeout 300 -p no:cacheprovider > $O/pytest.txt 2>&1
rc=$?
tail -3 $O/pytest.txt
[ $rc -ne 0 ] && exit $rc
EF_FIT_DEBUG=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/fr -o run -- python tools/prof_fit.py > $O/out.txt 2>&1 || exit $?
python tools/fit_breakdown.py /tmp/fr/run_kernel_trace.csv > $O/breakdown.txt && cp /tmp/fr/run_kernel_stats.csv $O/kernel_stats.csv
