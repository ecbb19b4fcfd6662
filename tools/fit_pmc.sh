#!/bin/bash
# Counters of the C3 fit's dominant kernels (SYRK, tall GEMMs): MFMA busy and clock.
# usage: bash tools/fit_pmc.sh <tag>
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/$1
mkdir -p $O
R="syrk|gemm_tall|chol_blk|tri_inv_blk|bj_round|transpose_stats|proj_i8|cov_finalize|gemm_s3"
timeout -s KILL 300 rocprofv3 --kernel-include-regex "$R" --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY --output-format csv -d $O/pmc_sq -o run -- python tools/prof_fit.py > $O/ps.txt 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --kernel-include-regex "$R" --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python tools/prof_fit.py > $O/pf.txt 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --kernel-include-regex "$R" --pmc TCC_HIT_sum TCC_MISS_sum SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD --output-format csv -d $O/pmc_l2 -o run -- python tools/prof_fit.py > $O/pl.txt 2>&1 || exit $?
python tools/pmc_kernels.py $O/pmc_sq/run_counter_collection.csv > $O/sq.txt
python tools/pmc_kernels.py $O/pmc_l2/run_counter_collection.csv > $O/l2.txt
python tools/pmc_kernels.py $O/pmc_fetch/run_counter_collection.csv > $O/fetch.txt
echo done
