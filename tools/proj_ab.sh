#!/bin/bash
# Training projection: 256- vs 128-column digit tiles (ef_proj_i8.hip).  Parity tests under
# both tile widths, then the C3 fit (+ projection) under the kernel tracer for each.
# usage: bash tools/proj_ab.sh <tag>
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_fit.py -x -q --timeout 200 -p no:cacheprovider > $O/pytest.txt 2>&1 || exit $?
for T in 128 256; do
  EF_LIB_VARIANT=diag EF_PROJ_TN=$T timeout -k 10 300 python -u -m pytest tests/test_gpu_fit.py -x -q --timeout 200 -p no:cacheprovider -k "projection or c3" > $O/pytest_tn$T.txt 2>&1 || exit $?
done
for T in 128 256; do
  EF_LIB_VARIANT=diag EF_PROJ_TN=$T timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_tn$T -o run -- python3 -u tools/proj_ab.py > $O/fit_tn$T.txt 2>&1 || exit $?
done
