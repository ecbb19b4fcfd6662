#!/bin/bash
# Round 6: gap-aware fit acceptance.  GPU tests of the fit (Dark / Light exact spectra,
# fixtures, the 1M C3 property test), then the C3 fit with the gap rule on and off
# (diagnostic build, EF_FIT_GAP_TOL=0 = round 5's rule): iterations, time, residual trace.
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${1:-r06/fitgap}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_manual.py tests/test_gpu_fit.py -s > $O/pytest.txt 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.txt; exit 1; }
grep -E "passed|failed|dark:|C3 1M" $O/pytest.txt
export EF_LIB_VARIANT=diag EF_FIT_DEBUG=1
for t in 1e-5 0; do
  EF_FIT_GAP_TOL=$t timeout -k 10 240 python tools/fit_ab.py $O/c3_$t.npz 5 > $O/c3_$t.txt 2>&1 || { echo "c3 rc=$?"; tail $O/c3_$t.txt; exit 1; }
  echo "C3 gap tol $t: $(grep 'rr it' $O/c3_$t.txt | tail -4 | tr '\n' ' ') $(grep median_s $O/c3_$t.txt)" >> $O/ab.txt
done
cat $O/ab.txt
