#!/bin/bash
# Round-5 closing run: the whole GPU suite, then the default bench line and the C3 fit
# breakdown on the final tree.
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${1:-r05/close}
mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
bash tools/r05_capture.sh ${1:-r05/close} bench && bash tools/r05_capture.sh ${1:-r05/close} fit
