#!/bin/bash
# C5 split-bf16 wide scan: HBM re-read experiment.  For the base library
# and variant libraries (tools/variant.sh: EF_WIDE3_PB probe tiles per XCD block,
# EF_WIDE_SERP serpentine k-slice order), the C5 bench line and one FETCH_SIZE pass of
# search_wide16_kernel.  usage: bash tools/c5_hbm_ab.sh <tag> <variant>...
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/$1; shift
mkdir -p $O
B="bench.py --config c5 --steps 3 --warmup 1 --repeats 1 --no-cpu --no-fit --no-image --no-split"
for v in base "$@"; do
  if [ "$v" = base ]; then unset EF_LIB_VARIANT; else export EF_LIB_VARIANT=$v; fi
  timeout -k 10 240 python bench.py --config c5 --no-cpu --no-fit --no-image --no-c2 --no-split --steps 10 \
    --repeats 3 > $O/$v.json 2> $O/$v.err || exit $?
  timeout -s KILL 180 rocprofv3 --kernel-include-regex search_wide16 --pmc FETCH_SIZE --output-format csv \
    -d $O/f_$v -o run -- python $B > $O/f_$v.txt 2>&1 || exit $?
  python - "$O" "$v" >> $O/summary.txt <<'PY'
import csv, json, sys
o, v = sys.argv[1], sys.argv[2]
d = json.loads(open(f"{o}/{v}.json").read().strip().splitlines()[-1])
rows = [r for r in csv.DictReader(open(f"{o}/f_{v}/run_counter_collection.csv")) if r.get("Counter_Name") == "FETCH_SIZE"]
per = {}
for r in rows:
    per.setdefault(r["Dispatch_Id"], 0.0)
    per[r["Dispatch_Id"]] += float(r["Counter_Value"])
vals = sorted(per.values())
med = vals[len(vals) // 2] if vals else float("nan")
print(v, d["value"], d["roofline"]["avg_launch_ms"], d["roofline"]["frac"], d["check"]["planted_match"],
      "FETCH_SIZE_kB_median", med, "x2_GB", round(2 * med * 1e3 / 1e9, 3), "launches", len(vals))
PY
done
echo done
