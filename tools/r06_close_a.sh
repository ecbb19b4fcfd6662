#!/bin/bash
# Round-6 closing run, part A: the whole GPU suite, smoke, the default bench line
cd "$GRAFT_REPO_ROOT" || exit 9
T=${1:-r06/close}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.txt 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke OK')" > $O/smoke.txt 2>&1 || { echo "smoke rc=$?"; tail $O/smoke.txt; exit 1; }
bash tools/r06_capture.sh $T bench
