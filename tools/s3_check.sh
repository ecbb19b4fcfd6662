#!/bin/bash
# Split-bf16 scan: parity tests, then the bench's headline + side leg, then a kernel trace
# of the split headline.  usage: bash tools/s3_check.sh <tag>
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_search_split.py tests/test_gpu_search.py > $O/pytest.out 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu --no-fit --no-image --no-c2 > $O/bench.out 2> $O/bench.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python bench.py --no-cpu --no-fit --no-image --no-c2 --no-split --search split_bf16 --steps 5 --repeats 2 \
  > $O/trace.out 2>&1 || exit $?
echo done
