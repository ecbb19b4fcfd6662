#!/bin/bash
# C5 bf16 projection check: projection parity tests, then the C5 bench line and a kernel
# trace (project_bf16_wide_kernel average).  usage: bash tools/proj_c5.sh <tag>
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_project.py -x -q --timeout 200 -p no:cacheprovider > $O/pytest.txt 2>&1
rc=$?
tail -3 $O/pytest.txt
[ $rc -ne 0 ] && exit $rc
B="bench.py --config c5 --steps 3 --warmup 1 --no-cpu --no-fit"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pc -o run -- python $B > $O/t.txt 2>&1 || exit $?
cp /tmp/pc/run_kernel_stats.csv $O/kernel_stats.csv
grep -E "project_bf16|search_wide" $O/kernel_stats.csv | cut -c1-160
