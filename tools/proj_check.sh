#!/bin/bash
# Projection change check: projection + search parity tests, then a short C3 bench.
# usage: bash tools/proj_check.sh <tag>
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${1:-pcheck}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_project.py tests/test_gpu_search.py tests/test_gpu_compat.py > $O/pytest.out 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu --no-fit --no-image > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 300 python bench.py --config c2 --steps 20 --warmup 3 --no-cpu --no-fit --no-image > $O/bench_c2.json 2> $O/bench_c2.err || exit $?
