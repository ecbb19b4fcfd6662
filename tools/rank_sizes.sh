#!/bin/bash
# Per-rank search efficiency at the strong-scaling shard sizes of C4 (1M rows / N ranks):
# one-GPU bench runs at 125k / 250k / 500k / 1M gallery rows.  usage: bash tools/rank_sizes.sh <tag>
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${1:-ranks}
mkdir -p $O
for g in 125000 250000 500000 1000000; do
  timeout -k 10 300 python bench.py --gallery $g --steps 20 --warmup 3 --no-cpu --no-fit --no-image --no-c2 --no-c5 \
    > $O/g$g.json 2> $O/g$g.err || exit $?
done
