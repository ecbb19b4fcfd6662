#!/bin/bash
# Block-Jacobi LDS-only barriers (product) vs __syncthreads (libeigenface_bjbar.so) on the
# C3 fit, alternated twice; results compared bit for bit; then the fit GPU tests.
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${1:-r05/bjbar}
mkdir -p $O
for rep in 1 2; do
  for v in product bjbar tsbar; do
    if [ $v = product ]; then unset EF_LIB_VARIANT; else export EF_LIB_VARIANT=$v; fi
    timeout -k 10 240 python tools/fit_ab.py $O/$v.npz 5 >> $O/ab.txt 2> $O/$v.$rep.err || { echo "$v rc=$?"; tail $O/$v.$rep.err; exit 1; }
  done
done
unset EF_LIB_VARIANT
python -c "
import numpy as np
a, b, c = np.load('$O/product.npz'), np.load('$O/bjbar.npz'), np.load('$O/tsbar.npz')
print('identical', all(np.array_equal(a[k], x[k]) for x in (b, c) for k in ('eigenvalues', 'components')))
" >> $O/ab.txt
cat $O/ab.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_fit.py tests/test_gpu_manual.py > $O/pytest.txt 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
