#!/bin/bash
# Blocked CholQR factor (csrc/ef_chol_blk.hip): microbenchmark against the register kernel
# (with a kernel trace splitting the factor and the inverse), then the C3 fit A/B against
# libeigenface_cholreg.so (-DEF_CHOL_REG: round 4's kernel), alternated twice.
# usage: bash tools/r05_chol.sh <tag> [skip-tests]
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${1:-r05/chol}
mkdir -p $O
timeout -k 10 60 tools/micro/bin/cib 256 128 88 200 > $O/cib.txt 2>&1 || { echo "cib rc=$?"; cat $O/cib.txt; exit 1; }
cat $O/cib.txt
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/cibprof -o run -- tools/micro/bin/cib 256 > $O/cibprof.txt 2>&1 || { echo "cibprof rc=$?"; exit 1; }
if [ -z "$2" ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_fit.py tests/test_gpu_manual.py tests/test_gpu_sharded_fit.py > $O/pytest.txt 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.txt; exit 1; }
  tail -3 $O/pytest.txt
fi
for rep in 1 2; do
  for v in product cholreg; do
    if [ $v = product ]; then unset EF_LIB_VARIANT; else export EF_LIB_VARIANT=$v; fi
    timeout -k 10 240 python tools/fit_ab.py $O/$v.npz 5 >> $O/ab.txt 2> $O/$v.$rep.err || { echo "fit_ab rc=$?"; tail $O/$v.$rep.err; exit 1; }
  done
done
cat $O/ab.txt
