#!/bin/bash
# fp32 coarse-phase switch threshold sweep on the C3 fit (diagnostic build, EF_FIT_DEBUG
# traces of every Rayleigh-Ritz step).  usage: bash tools/fit_tol.sh <tag>
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/$1
mkdir -p $O
for tol in 1e-4 1e-5 1e-6 1e-7 1e-4; do
  EF_LIB_VARIANT=diag EF_FIT_DEBUG=1 EF_FIT_COARSE_TOL=$tol timeout -k 10 200 python tools/prof_fit.py > $O/fit_$tol.txt 2>&1 || exit $?
  echo "tol=$tol $(grep -o "'gpu_fit_s': [0-9.]*" $O/fit_$tol.txt) $(grep -o "'eigensolver_iters': [0-9]*" $O/fit_$tol.txt) $(grep -o "'explained_variance_top3': [^]]*" $O/fit_$tol.txt)"
done
