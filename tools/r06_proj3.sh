#!/bin/bash
# Round 6: frag-form bf16 projection, round(mean) in LDS (ML) vs per-stage global mean loads:
# parity, alternated kernel traces, SQ / TA counters of the product form, FETCH/WRITE passes.
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${1:-r06/proj3}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_project.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.txt 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
B="bench.py --config c5 --steps 5 --warmup 2 --no-cpu --no-fit --no-split --no-image"
for v in ml1 ml0 ml1b ml0b; do
  case $v in ml1*) E=1;; ml0*) E=0;; esac
  EF_LIB_VARIANT=diag EF_PROJ_MEAN_LDS=$E timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$v -o run -- python $B > $O/t_$v.txt 2>&1 || { echo "trace rc=$?"; tail $O/t_$v.txt; exit 1; }
  python - $O/trace_$v/run_kernel_stats.csv $v <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'project_bf16' in r['Name']: print(sys.argv[2], r['Name'][:60], r['Calls'], r['AverageNs'])
PY
done
P="project_bf16_frag"
timeout -s KILL 180 rocprofv3 --kernel-include-regex "$P" --pmc FETCH_SIZE --output-format csv -d $O/proj_fetch -o run -- python $B > $O/qf.txt 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --kernel-include-regex "$P" --pmc WRITE_SIZE --output-format csv -d $O/proj_write -o run -- python $B > $O/qw.txt 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --kernel-include-regex "$P" --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS --output-format csv -d $O/proj_sq -o run -- python $B > $O/qs.txt 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --kernel-include-regex "$P" --pmc TA_BUSY_avr TCC_EA0_RDREQ_sum --output-format csv -d $O/proj_ta -o run -- python $B > $O/qt.txt 2>&1 || exit $?
python tools/pmc_kernels.py $O/proj_ta/run_counter_collection.csv > $O/ta.sum; cat $O/ta.sum
python tools/pmc_summary.py $O/proj_fetch/run_counter_collection.csv $O/proj_write/run_counter_collection.csv \
  $O/proj_sq/run_counter_collection.csv $O/trace_ml1/run_kernel_stats.csv $O/pmc_summary_c5proj.json c5proj || exit $?
cat $O/pmc_summary_c5proj.json
