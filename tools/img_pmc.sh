#!/bin/bash
# PMC passes (separate runs) over the image bench sections for the template-localiser and
# Haar kernels.  usage: bash tools/img_pmc.sh <tag>
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/$1
mkdir -p $O
R="tm_corr|haar_cascade"
timeout -s KILL 120 rocprofv3 --kernel-include-regex "$R" --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_LDS --output-format csv -d /tmp/ps -o run -- python tools/prof_image.py > $O/s.txt 2>&1 || exit $?
python tools/pmc_kernels.py /tmp/ps/run_counter_collection.csv > $O/sq.txt
timeout -s KILL 120 rocprofv3 --kernel-include-regex "$R" --pmc FETCH_SIZE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_INSTS_MFMA --output-format csv -d /tmp/pf -o run -- python tools/prof_image.py > $O/f.txt 2>&1 || exit $?
python tools/pmc_kernels.py /tmp/pf/run_counter_collection.csv > $O/fetch.txt
