#!/bin/bash
# Haar stage-group sweep: the Haar bench section per EF_HAAR_GROUPS setting (first stage of
# each group).  usage: bash tools/haar_groups.sh <tag> "1,3,6,10,15" "1,2,3,..." ...
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/$1; shift
mkdir -p $O
i=0
for g in "$@"; do
  i=$((i + 1))
  EF_HAAR_GROUPS=$g timeout -k 10 200 python -c "
import json, sys, torch
sys.path[:0] = ['.', 'face-detection-recognization-pca_amd']
import bench
from eigenface import Engine
torch.cuda.set_device(0)
e = Engine(0); e.timing(True)
r = [bench.haar_bench(e, False)['ms_per_frame_device'] for _ in range(3)]
print('$g', r, flush=True)
e.close()" >> $O/sweep.txt 2>&1 || exit $?
done
cat $O/sweep.txt
