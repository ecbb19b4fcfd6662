#!/bin/bash
# Search parity after a change to the scan kernels, the random-feature (unplanted) timings
# that exercise the collect pass, and the headline bench.  usage: bash tools/collect_check.sh <tag>
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_search.py tests/test_gpu_search_split.py tests/test_gpu_distributed.py tests/test_gpu_compat.py > $O/pytest.out 2>&1 || exit $?
for a in "512 0" "512 1" "128 0" "128 1"; do timeout -k 10 200 python tools/wide3_ablate.py $a >> $O/random.txt 2>&1 || exit $?; done
timeout -k 10 300 python bench.py --no-cpu --no-fit --no-image --no-c2 > $O/bench.out 2> $O/bench.err || exit $?
echo done
