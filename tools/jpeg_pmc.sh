#!/bin/bash
# PMC passes (separate runs) over the streamed JPEG ingest for the chunk kernels.
# usage: bash tools/jpeg_pmc.sh <tag>
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/$1
mkdir -p $O
R="jpeg_sync|jpeg_write|jpeg_idct|jpeg_resize"
timeout -s KILL 180 rocprofv3 --kernel-include-regex "$R" --pmc SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVE_CYCLES --output-format csv -d /tmp/jp1 -o run -- python tools/jpeg_async_prof.py > $O/p1.txt 2>&1 || exit $?
python tools/pmc_kernels.py /tmp/jp1/run_counter_collection.csv > $O/sq.txt
timeout -s KILL 180 rocprofv3 --kernel-include-regex "$R" --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY TA_BUSY_avr --output-format csv -d /tmp/jp2 -o run -- python tools/jpeg_async_prof.py > $O/p2.txt 2>&1 || exit $?
python tools/pmc_kernels.py /tmp/jp2/run_counter_collection.csv > $O/inst.txt
