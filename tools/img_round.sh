#!/bin/bash
# GPU image-side check: image/Haar parity tests, then the image bench sections under a
# rocprofv3 kernel trace.  usage: bash tools/img_round.sh <tag>
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_image.py tests/test_gpu_haar.py -x -q --timeout 300 -p no:cacheprovider > $O/pytest.txt 2>&1
rc=$?
tail -3 $O/pytest.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ir -o run -- python tools/prof_image.py > $O/out.txt 2>&1 || exit $?
cp /tmp/ir/run_kernel_stats.csv $O/kernel_stats.csv && grep -E "haar|Kernel_Name" /tmp/ir/run_kernel_trace.csv > $O/haar_trace.csv
