"""Aggregate a rocprofv3 --pmc counter_collection.csv per kernel: mean counter value per
dispatch.  usage: python tools/pmc_kernels.py <csv> [name-regex]"""
import collections
import csv
import re
import sys

pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
acc = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"]
    if pat and not pat.search(k):
        continue
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[k].add(r["Dispatch_Id"])
for k, cs in acc.items():
    n = len(disp[k])
    print(f"{k[:90]}  dispatches={n}")
    for c, v in sorted(cs.items()):
        print(f"    {c:28s} {v / n:.6g}")
