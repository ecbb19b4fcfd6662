#!/bin/bash
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
timeout -k 10 600 python -m pytest tests -m gpu -q --timeout 300 -p no:cacheprovider > gpurun_out/t2.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/t2.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > gpurun_out/bench2.json 2> gpurun_out/bench2.err
rc=$?; echo "bench rc=$rc" >> gpurun_out/bench2.err
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof2 -o run -- python bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/prof2.log 2>&1
echo "rocprof rc=$?" >> gpurun_out/prof2.log
