#!/bin/bash
# Split-bf16 scan counters: separate PMC passes of a headline run with the split scan.
# usage: bash tools/s3_pmc.sh <tag> [c3|c5]
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/$1
CFG=${2:-c3}
mkdir -p $O
B="bench.py --config $CFG --no-cpu --no-fit --no-image --no-c2 --no-split --search split_bf16 --steps 5 --warmup 2 --repeats 1"
R="search(16)?_(wide3_|wide16_)?kernel"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python $B > $O/t.txt 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --kernel-include-regex "$R" --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python $B > $O/pf.txt 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --kernel-include-regex "$R" --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python $B > $O/pw.txt 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --kernel-include-regex "$R" --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY --output-format csv -d $O/pmc_sq -o run -- python $B > $O/ps.txt 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --kernel-include-regex "$R" --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU --output-format csv -d $O/pmc_sq2 -o run -- python $B > $O/ps2.txt 2>&1 || exit $?
python tools/pmc_summary.py $O/pmc_fetch/run_counter_collection.csv $O/pmc_write/run_counter_collection.csv \
  $O/pmc_sq/run_counter_collection.csv $O/trace/run_kernel_stats.csv $O/pmc_summary_${CFG}s3.json ${CFG}s3 > /dev/null || exit $?
python tools/pmc_kernels.py $O/pmc_sq2/run_counter_collection.csv > $O/sq2.txt
echo done
