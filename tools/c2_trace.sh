#!/bin/bash
# Config 2 step (10k gallery, k = 64): kernel trace of the recognition step.
# usage: bash tools/c2_trace.sh <tag>
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python bench.py --config c2 --no-cpu --no-fit --no-image --no-split --steps 20 --repeats 2 > $O/c2.out 2>&1 || exit $?
echo done
