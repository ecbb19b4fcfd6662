#!/bin/bash
# Round 5: block-Jacobi early convergence test A/B on the C3 fit (product vs the
# EF_BJ_EARLY=0 variant libeigenface_bjold.so, alternated twice, results compared bit for
# bit), the fit parity tests, and the per-kernel breakdown of the C3 fit.
# usage: bash tools/r05_fit_ab.sh <tag>
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/$1
mkdir -p $O
for rep in 1 2; do
  for v in product bjold; do
    if [ $v = product ]; then unset EF_LIB_VARIANT; else export EF_LIB_VARIANT=$v; fi
    timeout -k 10 240 python tools/fit_ab.py $O/$v.npz 5 >> $O/ab.txt 2> $O/$v.$rep.err || exit $?
  done
done
unset EF_LIB_VARIANT
python -c "
import numpy as np
a, b = np.load('$O/product.npz'), np.load('$O/bjold.npz')
print('eigenvalues identical', bool(np.array_equal(a['eigenvalues'], b['eigenvalues'])),
      'components identical', bool(np.array_equal(a['components'], b['components'])),
      'max rel eig diff', float(np.max(np.abs(a['eigenvalues'] - b['eigenvalues']) / b['eigenvalues'])))
" >> $O/ab.txt || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_fit.py::test_device_tensors_outlive_a_closed_engine tests/test_gpu_sharded_fit.py tests/test_gpu_fit.py tests/test_gpu_manual.py -x -v --timeout 300 -p no:cacheprovider > $O/pytest.txt 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/fr -o run -- python tools/prof_fit.py > $O/prof.txt 2>&1 || exit $?
python tools/fit_breakdown.py /tmp/fr/run_kernel_trace.csv > $O/breakdown.txt && cp /tmp/fr/run_kernel_stats.csv $O/kernel_stats.csv
