#!/bin/bash
# One-term bf16 coarse products for the first iterations (EF_FIT_S1_ITERS, diagnostic
# build) on the C3 fit: iterations, sweeps, time, eigenvalue / component differences.
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${1:-r05/s1}
mkdir -p $O
export EF_LIB_VARIANT=diag EF_FIT_DEBUG=1
for rep in 1 2; do
  for n1 in 0 4 7 8; do
    EF_FIT_S1_ITERS=$n1 timeout -k 10 240 python tools/fit_ab.py $O/c3_$n1.npz 5 > $O/c3_$n1.txt 2>&1 || { echo "rc=$?"; tail $O/c3_$n1.txt; exit 1; }
    echo "S1 $n1 rep $rep: $(grep 'wide dim' $O/c3_$n1.txt | tail -1) $(grep median_s $O/c3_$n1.txt)" >> $O/ab.txt
  done
done
python - >> $O/ab.txt <<PY
import numpy as np
a = np.load("$O/c3_0.npz")
for n1 in (4, 7, 8):
    b = np.load(f"$O/c3_{n1}.npz")
    s = np.sign((a["components"] * b["components"]).sum(axis=1))
    print(n1, "eig rel", float(np.max(np.abs(a["eigenvalues"] - b["eigenvalues"]) / a["eigenvalues"])),
          "comp abs", float(np.max(np.abs(a["components"] - b["components"] * s[:, None]))))
PY
cat $O/ab.txt
