"""Per-kernel breakdown of the last full fit in a rocprofv3 kernel trace of tools/prof_fit.py.
usage: python tools/fit_breakdown.py <run_kernel_trace.csv>"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
first = [i for i, r in enumerate(rows) if "transpose_stats" in r["Kernel_Name"] or "shift_transpose" in r["Kernel_Name"]]
last = rows[first[-1]:]
t0 = int(last[0]["Start_Timestamp"])
agg = collections.defaultdict(lambda: [0, 0.0])
end = t0
for r in last:
    a = agg[r["Kernel_Name"][:80]]
    a[0] += 1
    a[1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    end = int(r["End_Timestamp"])
print(f"last fit (with training projection) span under the profiler {(end - t0) / 1e6:.1f} ms")
for k, v in sorted(agg.items(), key=lambda x: -x[1][1])[:16]:
    print(f"{v[1]:9.2f} ms {v[0]:6d}x  {k}")
