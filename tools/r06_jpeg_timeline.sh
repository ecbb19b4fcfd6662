#!/bin/bash
# device timeline of the streamed JPEG ingest (kernel + memory-copy trace, no counters)
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${1:-r06/jtl}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o run -- python tools/jpeg_timeline.py > $O/run.txt 2>&1 || { echo "rc=$?"; tail $O/run.txt; exit 1; }
grep wall $O/run.txt
python tools/jpeg_timeline_summary.py $O/trace/run_kernel_trace.csv $O/trace/run_memory_copy_trace.csv > $O/summary.txt
cat $O/summary.txt
