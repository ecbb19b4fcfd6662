#!/bin/bash
# Early Rayleigh-Ritz study at the C3 fit order (diagnostic build, EF_FIT_EARLY: 0 = product
# rule, 1 = iterations 1, 2, 4, n >= 2 = iteration n only): an early RR gives the spectral
# shift and the Chebyshev rate from that iteration on.  usage: bash tools/fit_early_probe.sh <tag>
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/$1
mkdir -p $O
for e in 0 1 2 3 4; do
  EF_LIB_VARIANT=diag EF_FIT_DEBUG=1 EF_FIT_EARLY=$e timeout -k 10 200 python tools/prof_fit.py > $O/e$e.txt 2>&1 || exit $?
  echo "early=$e $(grep -o "'gpu_fit_s': [0-9.]*" $O/e$e.txt) $(grep -o "'eigensolver_iters': [0-9]*" $O/e$e.txt) $(grep -o "'explained_variance_top3': \[[0-9., ]*" $O/e$e.txt) $(grep -c 'rr it' $O/e$e.txt) rr, sweeps $(grep 'rr it' $O/e$e.txt | tail -1 | grep -o 'sweeps_total=[0-9]*')" >> $O/summary.txt
done
echo done
