#!/bin/bash
# Round 6: frag-form bf16 projection with 4-wave workgroups, two per CU (EF_PROJ_NW=4,
# diagnostic build) vs the 8-wave product form: parity under both, alternated traces.
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${1:-r06/proj4}
mkdir -p $O
EF_LIB_VARIANT=diag EF_PROJ_NW=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_project.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_nw4.txt 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest_nw4.txt; exit 1; }
tail -1 $O/pytest_nw4.txt
B="bench.py --config c5 --steps 5 --warmup 2 --no-cpu --no-fit --no-split --no-image"
for v in nw8 nw4 nw8b nw4b; do
  case $v in nw8*) E=8;; nw4*) E=4;; esac
  EF_LIB_VARIANT=diag EF_PROJ_NW=$E timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$v -o run -- python $B > $O/t_$v.txt 2>&1 || { echo "trace rc=$?"; tail $O/t_$v.txt; exit 1; }
  python - $O/trace_$v/run_kernel_stats.csv $v <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'project_bf16' in r['Name'] or 'project_reduce' in r['Name']: print(sys.argv[2], r['Name'][:64], r['Calls'], r['AverageNs'])
PY
done
