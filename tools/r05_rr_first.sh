#!/bin/bash
# First Rayleigh-Ritz tolerance A/B on the C3 fit (diagnostic build, EF_FIT_RR_FIRST),
# alternated twice, with the eigensolver's sweep counts (EF_FIT_DEBUG).
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${1:-r05/rrfirst}
mkdir -p $O
export EF_LIB_VARIANT=diag EF_FIT_DEBUG=1
for rep in 1 2; do
  for t in 1e-4 1e-3 1e-2; do
    EF_FIT_RR_FIRST=$t timeout -k 10 240 python tools/fit_ab.py $O/t$t.npz 5 > $O/t$t.$rep.txt 2>&1 || { echo "rc=$?"; tail $O/t$t.$rep.txt; exit 1; }
    echo "tol $t rep $rep: $(grep sweeps= $O/t$t.$rep.txt | tail -1) $(grep median_s $O/t$t.$rep.txt)" >> $O/ab.txt
  done
done
python -c "
import numpy as np
a = np.load('$O/t1e-4.npz')
for t in ('1e-3', '1e-2'):
    b = np.load('$O/t%s.npz' % t)
    print(t, 'max rel eig diff', float(np.max(np.abs(a['eigenvalues'] - b['eigenvalues']) / a['eigenvalues'])))
" >> $O/ab.txt
cat $O/ab.txt
