#!/bin/bash
# Split-bf16 kernel shapes at C3: split tests, then the bench's split side leg with the
# 16x16x32 kernel (option 1) and the 32x32x16 one (option 2).  usage: bash tools/s3_ab.sh <tag>
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_search_split.py > $O/pytest.out 2>&1 || exit $?
B="bench.py --no-cpu --no-fit --no-image --no-c2"
timeout -k 10 300 python $B --split-opt 1 > $O/bench1.out 2> $O/bench1.err || exit $?
timeout -k 10 300 python $B --split-opt 2 > $O/bench2.out 2> $O/bench2.err || exit $?
timeout -k 10 300 python $B --split-opt 1 > $O/bench1b.out 2> $O/bench1b.err || exit $?
echo done
