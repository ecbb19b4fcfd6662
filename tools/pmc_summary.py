"""Summarise rocprofv3 --pmc passes of the search kernel into profiles/<round>/pmc_summary.json.

HBM bytes follow /opt/skills/guides/MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE
(KiB) from separate passes; on gfx950 FETCH_SIZE reports half the bytes of a wide
(16 B/lane) coalesced stream, so it is doubled; WRITE_SIZE is exact for 16-B stores
(the search kernel's partial-key stores are 8/4-B, uncalibrated: reported as is).
MFMA utilisation = SQ_VALU_MFMA_BUSY_CYCLES / (SIMDs x per-XCD GRBM_GUI_ACTIVE), the
clock = per-XCD GRBM_GUI_ACTIVE / kernel time.

usage: python tools/pmc_summary.py <fetch.csv> <write.csv> <sq.csv> <kernel_trace_stats.csv> <out.json> [config]
"""
import csv
import json
import sys
from collections import defaultdict

KERNEL = "search_kernel<128, 0, false, false, 0>"
# per config: (kernel name fragment, algorithmic bytes per launch = 4kN + 4N + 4kB)
CONFIGS = {
    "c3": ("search_kernel<128, 0, false, false, 0>", 1_000_000 * 128 * 4 + 1_000_000 * 4 + 4096 * 128 * 4),
    # split-bf16 scan: the split gallery copy has the fp32 gallery's bytes
    "c3s3": ("search16_kernel<0, false>", 1_000_000 * 128 * 4 + 1_000_000 * 4 + 4096 * 128 * 4),
    "c5s3": ("search_wide16_kernel<512, 0, false, false>", 1_000_000 * 512 * 4 + 1_000_000 * 4 + 4096 * 512 * 4),
    # the single-bf16 screen (EF_OPT_SEARCH_SPLIT_BF16 = 3): 2-byte gallery and probe copies,
    # launched with the row length in 4-byte units (KP = 512 / 2)
    "c5hi": ("search_wide16_kernel<256, 0, false, true>", 1_000_000 * 512 * 2 + 1_000_000 * 4 + 4096 * 512 * 2),
    # the 32x32x16 split wide kernel (EF_OPT_SEARCH_SPLIT_BF16 = 2)
    "c5s3w3": ("search_wide3_kernel<512, 0, false>", 1_000_000 * 512 * 4 + 1_000_000 * 4 + 4096 * 512 * 4),
    "c5": ("search_wide_kernel<512, 0, false>", 1_000_000 * 512 * 4 + 1_000_000 * 4 + 4096 * 512 * 4),
    # C5 bf16 projection: uint8 probe pixels + bf16 W + fp32 partial features
    "c5proj": ("project_bf16_frag_kernel", 4096 * 65536 + 512 * 65536 * 2 + 4096 * 512 * 4),
}
SIMDS = 1024  # 256 CUs x 4
XCDS = 8


def per_launch(path, kernel=KERNEL):
    acc = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if kernel in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}, {k: len(v) for k, v in acc.items()}


def avg_ns(stats_path, kernel=KERNEL):
    for r in csv.DictReader(open(stats_path)):
        if kernel in r["Name"]:
            return float(r["AverageNs"]), int(r["Calls"])
    raise SystemExit("kernel not found in stats")


def main():
    fetch, write, sq, stats, out = sys.argv[1:6]
    config = sys.argv[6] if len(sys.argv) > 6 else "c3"
    kernel, alg = CONFIGS[config]
    f, nf = per_launch(fetch, kernel)
    w, _ = per_launch(write, kernel)
    s, _ = per_launch(sq, kernel)
    ns, calls = avg_ns(stats, kernel)
    fetch_b = f["FETCH_SIZE"] * 1024 * 2  # gfx950: FETCH_SIZE counts half of wide reads
    write_b = w["WRITE_SIZE"] * 1024
    grbm_xcd = s["GRBM_GUI_ACTIVE"] / XCDS
    rec = {
        "config": config,
        "kernel": kernel,
        "launches_profiled": nf.get("FETCH_SIZE", 0),
        "fetch_size_kib_raw": f["FETCH_SIZE"],
        "write_size_kib_raw": w["WRITE_SIZE"],
        "hbm_read_bytes": fetch_b,
        "hbm_write_bytes": write_b,
        "traffic_bytes": fetch_b + write_b,
        "algorithmic_bytes": alg,
        "trace_avg_ns": ns,
        "trace_calls": calls,
        "mfma_busy_frac": s["SQ_VALU_MFMA_BUSY_CYCLES"] / (SIMDS * grbm_xcd),
        "clock_ghz": grbm_xcd / ns,
        "sq_wait_any_frac": s["SQ_WAIT_ANY"] / s["SQ_WAVE_CYCLES"],
    }
    if "SQ_LDS_BANK_CONFLICT" in s:
        rec["lds_bank_conflict_cycles"] = s["SQ_LDS_BANK_CONFLICT"]
        rec["lds_insts"] = s.get("SQ_INSTS_LDS")
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
