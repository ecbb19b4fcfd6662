#!/bin/bash
# Round 6 checkpoint: the whole -m gpu suite, then a kernel-trace breakdown of the C3 fit.
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/r06/full
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.txt 2>&1 || { echo "pytest rc=$?"; tail -40 $O/pytest_gpu.txt; exit 1; }
tail -3 $O/pytest_gpu.txt
bash tools/fit_prof.sh r06/fitprof
