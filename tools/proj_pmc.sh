#!/bin/bash
# Counters of the fp32 projection kernel on config 2 (k = 64) and config 3 (k = 128).
# usage: bash tools/proj_pmc.sh <tag>
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/$1
mkdir -p $O
for cfg in c2 c3; do
  B="bench.py --config $cfg --no-cpu --no-fit --no-image --no-c2 --no-split --steps 10 --warmup 2 --repeats 1"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$cfg -o run -- python $B > $O/t_$cfg.txt 2>&1 || exit $?
  timeout -s KILL 180 rocprofv3 --kernel-include-regex "project_kernel" --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS --output-format csv -d $O/pmc_$cfg -o run -- python $B > $O/p_$cfg.txt 2>&1 || exit $?
  python tools/pmc_kernels.py $O/pmc_$cfg/run_counter_collection.csv > $O/sq_$cfg.txt
done
echo done
