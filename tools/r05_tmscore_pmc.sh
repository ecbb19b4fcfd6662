#!/bin/bash
# Counters of the template localiser's score kernel on the bench frame.
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${1:-r05/tmscore_pmc}
mkdir -p $O
R="tm_score"
timeout -s KILL 120 rocprofv3 --kernel-include-regex "$R" --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --output-format csv -d $O/sq -o run -- python tools/prof_image.py > $O/sq.out 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-include-regex "$R" --pmc FETCH_SIZE TA_BUSY_avr GRBM_GUI_ACTIVE --output-format csv -d $O/ta -o run -- python tools/prof_image.py > $O/ta.out 2>&1 || exit $?
python tools/pmc_kernels.py $O/sq/run_counter_collection.csv > $O/summary.txt
python tools/pmc_kernels.py $O/ta/run_counter_collection.csv >> $O/summary.txt
cat $O/summary.txt
