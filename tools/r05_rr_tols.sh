#!/bin/bash
# Coarse Rayleigh-Ritz tolerances (diagnostic build): first step EF_FIT_RR_FIRST x later
# coarse steps EF_FIT_RR_LOOSE on the C3 fit and the C3-shape / C2-shape fits; iterations,
# sweeps, times and eigenvalue / component differences from the product defaults.
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${1:-r05/rrtols}
mkdir -p $O
export EF_LIB_VARIANT=diag EF_FIT_DEBUG=1 O
for cfg in "1e-2 1e-4" "1e-1 1e-4" "1e-2 1e-3" "1e-1 1e-3"; do
  set -- $cfg
  tag="f$1_l$2"
  EF_FIT_RR_FIRST=$1 EF_FIT_RR_LOOSE=$2 timeout -k 10 240 python tools/fit_ab.py $O/c3_$tag.npz 5 > $O/c3_$tag.txt 2>&1 || { echo "c3 rc=$?"; tail $O/c3_$tag.txt; exit 1; }
  echo "C3 $tag: $(grep 'wide dim' $O/c3_$tag.txt | tail -1) $(grep median_s $O/c3_$tag.txt)" >> $O/ab.txt
  TAG=$tag EF_FIT_RR_FIRST=$1 EF_FIT_RR_LOOSE=$2 timeout -k 10 300 python - > $O/small_$tag.txt 2>&1 <<'PY' || { echo "small rc=$?"; tail $O/small_$tag.txt; exit 1; }
import sys, time, os
sys.path.insert(0, "face-detection-recognization-pca_amd"); sys.path.insert(0, ".")
import numpy as np, torch
from oracle import eigenface_oracle as orc
from eigenface import Engine
eng = Engine(0)
tag = os.environ["TAG"]
for n, side, k, std in ((10000, 128, 64, False), (20000, 128, 128, True)):
    x, _ = orc.synth_faces(n, side, r=256, seed=n)
    xd = torch.from_numpy(x).cuda()
    eng.fit(xd, k, standardize=std, projection=False)
    ts = []
    for _ in range(3):
        torch.cuda.synchronize(); t = time.perf_counter()
        r = eng.fit(xd, k, standardize=std, projection=False)
        torch.cuda.synchronize(); ts.append(time.perf_counter() - t)
    np.savez(f"{os.environ['O']}/small_{tag}_{n}.npz", ev=r.eigenvalues.cpu().numpy(), comps=r.components.cpu().numpy())
    print("n", n, "median_s", round(float(np.median(ts)), 4), "iters", r.iters, flush=True)
PY
  grep -E "median_s" $O/small_$tag.txt | sed "s/^/small $tag: /" >> $O/ab.txt
done
python - >> $O/ab.txt <<PY
import numpy as np
def cmp(a, b):
    ea, eb = (a["ev"] if "ev" in a.files else a["eigenvalues"]), (b["ev"] if "ev" in b.files else b["eigenvalues"])
    ca, cb = (a["comps"] if "comps" in a.files else a["components"]), (b["comps"] if "comps" in b.files else b["components"])
    s = np.sign((ca * cb).sum(axis=1))
    return float(np.max(np.abs(ea - eb) / np.abs(ea))), float(np.max(np.abs(ca - cb * s[:, None])))
base = "f1e-2_l1e-4"
for t in ("f1e-1_l1e-4", "f1e-2_l1e-3", "f1e-1_l1e-3"):
    print("C3", t, "vs", base, cmp(np.load(f"$O/c3_{base}.npz"), np.load(f"$O/c3_{t}.npz")))
    for n in (10000, 20000):
        print("small", n, t, cmp(np.load(f"$O/small_{base}_{n}.npz"), np.load(f"$O/small_{t}_{n}.npz")))
PY
cat $O/ab.txt
