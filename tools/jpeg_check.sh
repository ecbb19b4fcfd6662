#!/bin/bash
# JPEG path: decode/ingest tests, then the bench's JPEG line and the stage profile.
# usage: bash tools/jpeg_check.sh <tag>
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_jpeg.py tests/test_gpu_search_split.py > $O/pytest.out 2>&1 || exit $?
timeout -k 10 300 python tools/micro/jpeg_prof.py > $O/prof.txt 2>&1 || exit $?
timeout -k 10 300 python -c "
import sys, json; sys.path[:0] = ['.', 'face-detection-recognization-pca_amd']
import torch; torch.cuda.init()
import bench
from eigenface import Engine
e = Engine(0); e.timing(True)
sides = [s for g in bench.TEMPLATE_SIDES for s in g]
print(json.dumps(bench.jpeg_ingest_bench(e, False, sides)))
" > $O/jbench.out 2>&1 || exit $?
echo done
