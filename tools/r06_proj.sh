#!/bin/bash
# Round 6: frag-form bf16 projection (W16 in MFMA-fragment order, B operand straight from
# L2 into VGPRs).  Projection parity tests, then the C5 step under a kernel trace with the
# product library (frag form) and the diagnostic library with EF_PROJ_FRAG=0 (round 5's
# wide kernel), then FETCH/WRITE/SQ passes of the frag kernel.   usage: bash tools/r06_proj.sh <tag>
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${1:-r06/proj}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_project.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.txt 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
B="bench.py --config c5 --steps 5 --warmup 2 --no-cpu --no-fit --no-split --no-image"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_frag -o run -- python $B > $O/t_frag.txt 2>&1 || { echo "trace rc=$?"; tail $O/t_frag.txt; exit 1; }
EF_LIB_VARIANT=diag EF_PROJ_FRAG=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_wide -o run -- python $B > $O/t_wide.txt 2>&1 || { echo "trace rc=$?"; tail $O/t_wide.txt; exit 1; }
grep -hE "project_bf16|search_wide16|project_reduce" $O/trace_frag/run_kernel_stats.csv $O/trace_wide/run_kernel_stats.csv | cut -d, -f1-6
P="project_bf16_frag"
timeout -s KILL 180 rocprofv3 --kernel-include-regex "$P" --pmc FETCH_SIZE --output-format csv -d $O/proj_fetch -o run -- python $B > $O/qf.txt 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --kernel-include-regex "$P" --pmc WRITE_SIZE --output-format csv -d $O/proj_write -o run -- python $B > $O/qw.txt 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --kernel-include-regex "$P" --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS --output-format csv -d $O/proj_sq -o run -- python $B > $O/qs.txt 2>&1 || exit $?
python tools/pmc_summary.py $O/proj_fetch/run_counter_collection.csv $O/proj_write/run_counter_collection.csv \
  $O/proj_sq/run_counter_collection.csv $O/trace_frag/run_kernel_stats.csv $O/pmc_summary_c5proj.json c5proj || exit $?
cat $O/pmc_summary_c5proj.json
