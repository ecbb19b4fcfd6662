#!/bin/bash
# SYRK16 stage tail: one column after the barrier (product) vs two (libeigenface_s16t2.so,
# EF_S16_TAIL=2), C3 fit alternated twice, results compared bit for bit (integer SYRK).
# usage: bash tools/r05_syrk_tail.sh <tag> [variant]
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/$1
V=${2:-s16t2}
mkdir -p $O
for rep in 1 2; do
  for v in product $V; do
    if [ $v = product ]; then unset EF_LIB_VARIANT; else export EF_LIB_VARIANT=$v; fi
    timeout -k 10 240 python tools/fit_ab.py $O/$v.npz 5 >> $O/ab.txt 2> $O/$v.$rep.err || exit $?
  done
done
unset EF_LIB_VARIANT
python -c "
import numpy as np
a, b = np.load('$O/product.npz'), np.load('$O/$V.npz')
print('eigenvalues identical', bool(np.array_equal(a['eigenvalues'], b['eigenvalues'])))
" >> $O/ab.txt
cat $O/ab.txt
