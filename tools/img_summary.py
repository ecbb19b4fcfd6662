"""Summarise the image-side rocprofv3 passes (tools/r05_capture.sh part `image`) into
profiles/<round>/pmc_summary_tmatch.json and pmc_summary_haar.json.

  tmatch: tm_corr_kernel (the template localiser's int8 MFMA correlation): MFMA busy
          fraction of SIMD-cycles, clock, HBM bytes (FETCH_SIZE x2 + WRITE_SIZE is not
          collected: the kernel reads L2-resident frame rows and bands), LDS bank conflicts.
  haar:   haar_cascade_split_kernel (the gather-bound stage groups): TA busy fraction
          = TA_BUSY_avr / per-XCD GRBM_GUI_ACTIVE — the texture-address unit every
          integral-image gather passes through, the kernel's bound (DESIGN K12).

usage: python tools/img_summary.py <sq.csv> <ta.csv> <kernel_stats.csv> <out_dir>
"""
import csv
import json
import os
import sys
from collections import defaultdict

SIMDS, XCDS = 1024, 8


def per_kernel(path, frag):
    acc, disp = defaultdict(float), set()
    for r in csv.DictReader(open(path)):
        if frag in r["Kernel_Name"]:
            acc[r["Counter_Name"]] += float(r["Counter_Value"])
            disp.add(r["Dispatch_Id"])
    n = max(len(disp), 1)
    return {k: v / n for k, v in acc.items()}, len(disp)


def trace(stats, frag):
    tot, calls = 0.0, 0
    for r in csv.DictReader(open(stats)):
        if frag in r["Name"]:
            tot += float(r["TotalDurationNs"])
            calls += int(r["Calls"])
    return (tot / calls if calls else None), calls


def main():
    sq, ta, stats, out_dir = sys.argv[1:5]
    os.makedirs(out_dir, exist_ok=True)
    s, n = per_kernel(sq, "tm_corr_kernel")
    ns, calls = trace(stats, "tm_corr_kernel")
    g = s["GRBM_GUI_ACTIVE"] / XCDS
    tm = {"config": "tmatch", "kernel": "tm_corr_kernel", "dispatches_profiled": n, "trace_avg_ns": ns,
          "trace_calls": calls, "mfma_busy_frac": s["SQ_VALU_MFMA_BUSY_CYCLES"] / (SIMDS * g),
          "clock_ghz": g / ns if ns else None, "sq_wait_any_frac": s["SQ_WAIT_ANY"] / s["SQ_WAVE_CYCLES"],
          "lds_bank_conflict_cycles": s.get("SQ_LDS_BANK_CONFLICT")}
    t, nt = per_kernel(ta, "haar_cascade_split_kernel")
    hns, hcalls = trace(stats, "haar_cascade_split_kernel")
    gt = t["GRBM_GUI_ACTIVE"] / XCDS
    haar = {"config": "haar", "kernel": "haar_cascade_split_kernel", "dispatches_profiled": nt,
            "trace_avg_ns": hns, "trace_calls": hcalls, "ta_busy_frac": t["TA_BUSY_avr"] / gt,
            "fetch_size_kib_raw": t.get("FETCH_SIZE"), "clock_ghz": gt / hns if hns else None}
    for name, rec in (("pmc_summary_tmatch.json", tm), ("pmc_summary_haar.json", haar)):
        json.dump(rec, open(os.path.join(out_dir, name), "w"), indent=1)
        print(json.dumps(rec))


if __name__ == "__main__":
    main()
