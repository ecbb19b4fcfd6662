"""Per-dispatch durations from a rocprofv3 kernel_trace.csv: for each kernel name, the
durations in launch order (first N) — e.g. the JPEG sync rounds of one decode."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 12
by = defaultdict(list)
for r in rows:
    by[r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][-40:]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in by.items():
    print(f"{k:40s} n={len(v):4d} " + " ".join(f"{x:.0f}" for x in v[:n]))
