#!/bin/bash
# Phase stamps of tm_corr_kernel on the bench's 640x480 x 60-map frame (EF_TM_STAMP build,
# libeigenface_tmstamp.so): per k-block count, the share of each wave's loop time spent
# issuing fragment reads + MFMAs (+ interleaved DMA), waiting for the DMA, and in the barrier.
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${1:-r05/tmstamp}
mkdir -p $O
EF_LIB_VARIANT=${2:-tmstamp} timeout -k 10 200 python -u tools/prof_image.py > $O/run.txt 2> $O/run.err || { echo "rc=$?"; tail -5 $O/run.err; exit 1; }
python - $O/run.txt > $O/summary.txt <<'PY'
import re, sys
from collections import defaultdict
acc = defaultdict(lambda: [0, 0, 0, 0, 0, 0])
for l in open(sys.argv[1]):
    m = re.search(r"tmstamp blk \d+ wave (\d+) nkb (\d+) pairs (\d+) issue (\d+) mfma (\d+) vmwait (\d+) barrier (\d+)", l)
    if m:
        w, nkb, pairs, *ph = map(int, m.groups())
        a = acc[nkb]
        a[0] += 1; a[1] += pairs
        for i in range(4):
            a[2 + i] += ph[i]
print("nkb samples pairs  cyc/pair  mfma%  vmwait%  barrier%  other%")
for nkb in sorted(acc):
    n, pairs, i0, mf, vw, br = acc[nkb]
    tot = i0 + mf + vw + br
    print(f"{nkb:3d} {n:7d} {pairs:6d} {tot / pairs:9.0f} {100 * mf / tot:6.1f} {100 * vw / tot:8.1f} {100 * br / tot:9.1f} {100 * i0 / tot:7.1f}")
PY
cat $O/summary.txt
