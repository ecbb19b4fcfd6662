#!/bin/bash
# Config 5 with the split-bf16 scan: wide split tests, C5 bench (fp32 headline + split leg),
# kernel trace of the split run.  usage: bash tools/c5s3.sh <tag>
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_search_split.py > $O/pytest.out 2>&1 || exit $?
timeout -k 10 300 python bench.py --config c5 --steps 5 --warmup 2 --no-cpu --no-fit --no-image > $O/bench.out 2> $O/bench.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python bench.py --config c5 --no-cpu --no-fit --no-image --no-split --search split_bf16 --steps 3 --repeats 1 \
  > $O/trace.out 2>&1 || exit $?
echo done
