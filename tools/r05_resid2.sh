#!/bin/bash
# Ritz-residual acceptance as the default: every fit / manual / sharded-fit GPU test, the
# drop-in and compat tests (the trainers fit through the same solver), and the C3 fit.
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${1:-r05/resid2}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_fit.py tests/test_gpu_manual.py tests/test_gpu_sharded_fit.py tests/test_gpu_dropin.py tests/test_gpu_compat.py > $O/pytest.txt 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
timeout -k 10 240 python tools/fit_ab.py /tmp/p.npz 5 > $O/fit.txt 2>&1 || { echo "fit rc=$?"; tail $O/fit.txt; exit 1; }
cat $O/fit.txt
