#!/bin/bash
# Round 6: the screen epilogue on raw accumulators (L2: skip test on -2 max(a), values
# scaled only in blocks that pass it) vs the previous tree's (libeigenface_prev.so, built
# from the previous ef_search_wide.hip), alternated under a kernel trace; then the parity tests.
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${1:-r06/screenraw}
mkdir -p $O
B="bench.py --config c5 --split-opt 3 --steps 10 --warmup 2 --repeats 3 --no-cpu --no-fit --no-split --no-image"
for v in new prev newb prevb; do
  case $v in new*) L="";; prev*) L="prev";; esac
  EF_LIB_VARIANT=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$v -o run -- python $B > $O/t_$v.txt 2>&1 || { echo "trace rc=$?"; tail $O/t_$v.txt; exit 1; }
  python - $O/trace_$v/run_kernel_stats.csv $v <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'search_wide16' in r['Name']: print(sys.argv[2], r['Name'][:60], r['Calls'], r['AverageNs'])
PY
  python -c "
import json
r=json.loads([l for l in open('$O/t_$v.txt') if l.startswith('{')][-1])
print('$v', 'ms_per_step', r['ms_per_step'], 'value', r['value'], 'planted', r.get('check'))"
done
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_c5_full.py tests/test_gpu_search_split.py > $O/pytest.txt 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
