#!/bin/bash
# C5 wide-search capture: bench line, kernel trace, separate PMC passes (FETCH_SIZE /
# WRITE_SIZE / SQ) -> pmc_summary_c5.json, plus diagnostic passes (LDS, L2 hit).
# usage: bash tools/c5_pmc.sh <tag>
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/$1
mkdir -p $O
# the C5 headline scan is the split-bf16 one (search_wide16_kernel); the fp32 wide kernel is
# the bench's side leg (its r02 PMC summary stays in profiles/r02/pmc_summary_c5.json)
# SPLIT=3 (default): the single-bf16 screen (pmc_summary_c5hi.json); SPLIT=1: the split-bf16 scan
SPLIT=${SPLIT:-3}
CFG=$([ "$SPLIT" = 3 ] && echo c5hi || echo c5s3)
B="bench.py --config c5 --split-opt $SPLIT --steps 3 --warmup 1 --no-cpu --no-fit --no-split --no-image"
R="search_wide16"
timeout -k 10 300 python bench.py --config c5 --split-opt $SPLIT --steps 5 --warmup 2 --no-cpu --no-fit > $O/bench.txt 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python $B > $O/t.txt 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --kernel-include-regex "$R" --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python $B > $O/pf.txt 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --kernel-include-regex "$R" --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python $B > $O/pw.txt 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --kernel-include-regex "$R" --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY --output-format csv -d $O/pmc_sq -o run -- python $B > $O/ps.txt 2>&1 || exit $?
python tools/pmc_summary.py $O/pmc_fetch/run_counter_collection.csv $O/pmc_write/run_counter_collection.csv \
  $O/pmc_sq/run_counter_collection.csv $O/trace/run_kernel_stats.csv $O/pmc_summary_$CFG.json $CFG > /dev/null || exit $?
timeout -s KILL 180 rocprofv3 --kernel-include-regex "$R" --pmc TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d /tmp/ph -o run -- python $B > $O/h.txt 2>&1 || exit $?
python tools/pmc_kernels.py /tmp/ph/run_counter_collection.csv > $O/l2.txt
# bf16 projection: the same passes for project_bf16_wide_kernel
P="project_bf16_frag"
timeout -s KILL 180 rocprofv3 --kernel-include-regex "$P" --pmc FETCH_SIZE --output-format csv -d $O/proj_fetch -o run -- python $B > $O/qf.txt 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --kernel-include-regex "$P" --pmc WRITE_SIZE --output-format csv -d $O/proj_write -o run -- python $B > $O/qw.txt 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --kernel-include-regex "$P" --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS --output-format csv -d $O/proj_sq -o run -- python $B > $O/qs.txt 2>&1 || exit $?
python tools/pmc_summary.py $O/proj_fetch/run_counter_collection.csv $O/proj_write/run_counter_collection.csv \
  $O/proj_sq/run_counter_collection.csv $O/trace/run_kernel_stats.csv $O/pmc_summary_c5proj.json c5proj || exit $?
