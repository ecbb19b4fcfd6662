#!/bin/bash
# Copy one tools/gpu_round.sh output set (gpurun_out/<tag>) into profiles/<round>/.
# usage: bash tools/save_profiles.sh <tag> <round-dir>
set -e
O=gpurun_out/$1; P=profiles/$2
mkdir -p $P
cp $O/trace/run_kernel_stats.csv $P/kernel_stats.csv
cp $O/pmc_fetch/run_counter_collection.csv $P/pmc_fetch_counters.csv
cp $O/pmc_write/run_counter_collection.csv $P/pmc_write_counters.csv
cp $O/pmc_sq/run_counter_collection.csv $P/pmc_sq_counters.csv
tail -1 $O/bench.out > $P/bench.json
tail -3 $O/pytest.out > $P/pytest_gpu.txt
python tools/pmc_summary.py $O/pmc_fetch/run_counter_collection.csv $O/pmc_write/run_counter_collection.csv \
  $O/pmc_sq/run_counter_collection.csv $O/trace/run_kernel_stats.csv $P/pmc_summary.json > /dev/null
