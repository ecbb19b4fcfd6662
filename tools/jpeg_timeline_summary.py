"""Per-batch device timeline of tools/jpeg_timeline.py's trace: batch period (first kernel
to first kernel), kernel-busy time, idle gaps and what precedes each gap.
usage: python tools/jpeg_timeline_summary.py <kernel_trace.csv> <memory_copy_trace.csv>"""
import csv
import sys

ks = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
cps = sorted(csv.DictReader(open(sys.argv[2])), key=lambda r: int(r["Start_Timestamp"])) if len(sys.argv) > 2 else []
ks = [r for r in ks if "jpeg" in r["Kernel_Name"] or "rocclr" in r["Kernel_Name"]]
starts = [i for i, r in enumerate(ks) if "jpeg_sync_kernel" in r["Kernel_Name"]]
# batch = run of kernels starting at the first sync kernel after a non-sync kernel
bstarts = [i for i in starts if i == 0 or "jpeg_sync_kernel" not in ks[i - 1]["Kernel_Name"]]
bstarts = bstarts[-16:]
print(f"{len(bstarts)} batches analysed")
for a, b in zip(bstarts, bstarts[1:]):
    seg = ks[a:b]
    t0, t1 = int(seg[0]["Start_Timestamp"]), int(ks[b]["Start_Timestamp"])
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg)
    gaps = []
    for x, y in zip(seg, seg[1:] + [ks[b]]):
        g = int(y["Start_Timestamp"]) - int(x["End_Timestamp"])
        if g > 20000:
            gaps.append(f"{g / 1e3:.0f}us before {y['Kernel_Name'][:28]}")
    cp = [c for c in cps if t0 <= int(c["Start_Timestamp"]) < t1]
    cpt = sum(int(c["End_Timestamp"]) - int(c["Start_Timestamp"]) for c in cp)
    print(f"period {(t1 - t0) / 1e6:.3f} ms  kernels {busy / 1e6:.3f} ms  n={len(seg)}  copies {len(cp)} "
          f"({cpt / 1e6:.3f} ms)  gaps: {'; '.join(gaps)}")
