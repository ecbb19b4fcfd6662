#!/bin/bash
# Round 6: gallery-in-VGPRs screen, 64-B-contiguous gallery loads: parity (screen cases),
# C5 step A/B vs search_wide16_kernel (alternated), and SQ / TA counters of both.
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${1:-r06/screen2}
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_search_split.py > $O/pytest_split.txt 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest_split.txt; exit 1; }
tail -1 $O/pytest_split.txt
B="bench.py --config c5 --split-opt 3 --steps 10 --warmup 2 --repeats 3 --no-cpu --no-fit --no-split --no-image"
for v in vg1 vg0 vg1b; do
  case $v in vg1*) E=1;; vg0*) E=0;; esac
  EF_LIB_VARIANT=diag EF_SCREEN_VG=$E timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$v -o run -- python $B > $O/t_$v.txt 2>&1 || { echo "trace rc=$?"; tail $O/t_$v.txt; exit 1; }
  python - $O/trace_$v/run_kernel_stats.csv $v <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'search_screen' in r['Name'] or 'search_wide16' in r['Name']: print(sys.argv[2], r['Name'][:70], r['Calls'], r['AverageNs'])
PY
done
B2="bench.py --config c5 --split-opt 3 --steps 3 --warmup 1 --repeats 1 --no-cpu --no-fit --no-split --no-image"
for v in 1 0; do
  EF_LIB_VARIANT=diag EF_SCREEN_VG=$v timeout -s KILL 180 rocprofv3 --kernel-include-regex "search_screen|search_wide16_kernel<256, 0, false" --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS --output-format csv -d $O/sq_$v -o run -- python $B2 > $O/sq_$v.txt 2>&1 || exit $?
  python tools/pmc_kernels.py $O/sq_$v/run_counter_collection.csv > $O/sq_$v.sum; cat $O/sq_$v.sum
  EF_LIB_VARIANT=diag EF_SCREEN_VG=$v timeout -s KILL 180 rocprofv3 --kernel-include-regex "search_screen|search_wide16_kernel<256, 0, false" --pmc TA_BUSY_avr FETCH_SIZE --output-format csv -d $O/ta_$v -o run -- python $B2 > $O/ta_$v.txt 2>&1 || exit $?
  python tools/pmc_kernels.py $O/ta_$v/run_counter_collection.csv > $O/ta_$v.sum; cat $O/ta_$v.sum
done
