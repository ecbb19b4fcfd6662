#!/bin/bash
# Round 6: C2 at its own size (tests/test_gpu_c2_full.py) and the k = 64 fp32 projection's
# branch-free FAST form against the generic one (diagnostic build, EF_PROJ_FAST=0): the
# bench's c2 record (projection avg launch ms and fraction of fp32 peak) for each.
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${1:-r06/c2}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_c2_full.py tests/test_gpu_project.py -s > $O/pytest.txt 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
B="bench.py --steps 5 --warmup 2 --repeats 3 --no-cpu --no-fit --no-c5 --no-image --no-split"
for v in prod fast0; do
  if [ $v = fast0 ]; then export EF_LIB_VARIANT=diag EF_PROJ_FAST=0; fi
  timeout -k 10 300 python $B > $O/bench_$v.txt 2>&1 || { echo "bench rc=$?"; tail $O/bench_$v.txt; exit 1; }
  python -c "
import json,sys
r=json.loads([l for l in open('$O/bench_$v.txt') if l.startswith('{')][-1])
c=r['c2']; print('$v', c['ms_per_step'], c['roofline']['avg_launch_ms'], c['roofline']['frac'], c['roofline']['search'])"
done
