#!/bin/bash
# Coarse-phase switch study (diagnostic build): the C3 fit's Rayleigh-Ritz trajectory
# (EF_FIT_DEBUG) at the default switch and with later switches (EF_FIT_COARSE_TOL /
# EF_FIT_COARSE_PRED), fit seconds and top eigenvalues.  usage: bash tools/fit_coarse_probe.sh <tag>
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/$1
mkdir -p $O
run() {  # name, tol, pred
  EF_LIB_VARIANT=diag EF_FIT_DEBUG=1 EF_FIT_COARSE_TOL=$2 EF_FIT_COARSE_PRED=$3 timeout -k 10 200 \
    python tools/prof_fit.py > $O/$1.txt 2>&1 || exit $?
  echo "$1 $(grep -o "'gpu_fit_s': [0-9.]*" $O/$1.txt) $(grep -o "'eigensolver_iters': [0-9]*" $O/$1.txt)" >> $O/summary.txt
}
run default 1e-4 1e-6
run t6 1e-6 1e-8
run t8 1e-8 1e-10
run t10 1e-10 1e-12
echo done
