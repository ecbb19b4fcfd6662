#!/bin/bash
# Copy one tools/final_round.sh capture (gpurun_out/<tag>*) into profiles/<round>/.
# usage: bash tools/save_round.sh <tag> <round-dir>
set -e
T=$1; P=profiles/$2
bash tools/save_profiles.sh $T $2
C=gpurun_out/${T}_c5
tail -1 $C/bench.txt > $P/bench_c5.json
cp $C/trace/run_kernel_stats.csv $P/c5_kernel_stats.csv
cp $C/pmc_fetch/run_counter_collection.csv $P/c5_pmc_fetch_counters.csv
cp $C/pmc_write/run_counter_collection.csv $P/c5_pmc_write_counters.csv
cp $C/pmc_sq/run_counter_collection.csv $P/c5_pmc_sq_counters.csv
cp $C/proj_fetch/run_counter_collection.csv $P/c5proj_pmc_fetch_counters.csv
cp $C/proj_write/run_counter_collection.csv $P/c5proj_pmc_write_counters.csv
cp $C/proj_sq/run_counter_collection.csv $P/c5proj_pmc_sq_counters.csv
cp $C/pmc_summary_c5proj.json $P/
if [ -f $C/pmc_summary_c5hi.json ]; then  # c5_pmc.sh default: the single-bf16 screen
  cp $C/pmc_summary_c5hi.json $P/ && cp $C/l2.txt $P/c5hi_l2_counters.txt
else
  cp $C/pmc_summary_c5s3.json $P/ && cp $C/l2.txt $P/c5_l2_counters.txt
fi
cp gpurun_out/${T}_fit/breakdown.txt $P/fit_c3_breakdown.txt
cp gpurun_out/${T}_fit/kernel_stats.csv $P/fit_c3_kernel_stats.csv
cp gpurun_out/${T}_img/kernel_stats.csv $P/image_kernel_stats.csv
cp gpurun_out/${T}_img/haar_trace.csv $P/haar_trace.csv
