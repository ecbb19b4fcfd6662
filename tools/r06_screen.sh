#!/bin/bash
# Round 6: the gallery-in-VGPRs screen (ef_search_screen.hip) — parity
# tests, then the C5 step A/B against search_wide16_kernel's main pass (diagnostic build,
# EF_SCREEN_VG=0), alternated, under a kernel trace.   usage: bash tools/r06_screen.sh <tag>
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${1:-r06/screen}
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_search_split.py > $O/pytest_split.txt 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest_split.txt; exit 1; }
tail -1 $O/pytest_split.txt
B="bench.py --config c5 --split-opt 3 --steps 10 --warmup 2 --repeats 3 --no-cpu --no-fit --no-split --no-image"
for v in vg1 vg0 vg1b vg0b; do
  case $v in vg1*) E=1;; vg0*) E=0;; esac
  EF_LIB_VARIANT=diag EF_SCREEN_VG=$E timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$v -o run -- python $B > $O/t_$v.txt 2>&1 || { echo "trace rc=$?"; tail $O/t_$v.txt; exit 1; }
  python - $O/trace_$v/run_kernel_stats.csv $v <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'search_screen' in r['Name'] or 'search_wide16' in r['Name']: print(sys.argv[2], r['Name'][:70], r['Calls'], r['AverageNs'])
PY
  python -c "
import json
r=json.loads([l for l in open('$O/t_$v.txt') if l.startswith('{')][-1])
print('$v', 'ms_per_step', r['ms_per_step'], 'value', r['value'], 'planted', r.get('check'))"
done
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_c5_full.py > $O/pytest_c5.txt 2>&1 || { echo "pytest c5 rc=$?"; tail -30 $O/pytest_c5.txt; exit 1; }
tail -1 $O/pytest_c5.txt
