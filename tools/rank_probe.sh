#!/bin/bash
# 125k-row shard (C4 at N=8): kernel trace vs hipEvent timing, and workgroup-count variants.
# usage: bash tools/rank_probe.sh <tag>
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${1:-rprobe}
mkdir -p $O
B="bench.py --gallery 125000 --steps 20 --warmup 3 --no-cpu --no-fit --no-image"
for w in 256 512 1024; do
  EF_SEARCH_WGS=$w timeout -k 10 300 python $B > $O/wgs$w.json 2> $O/wgs$w.err || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python $B \
  > $O/trace.out 2> $O/trace.err || exit $?
