#!/bin/bash
# Template localiser score kernel: kernel trace of the bench frame for the product library
# and variant libraries (e.g. tmscoreabl = no fp64 normalisation, results invalid).
# usage: bash tools/r05_tmscore.sh <tag> <variant>...
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
TAG=${1:-r05/tmscore}; shift
O=gpurun_out/$TAG
mkdir -p $O
for v in product "$@"; do
  if [ $v = product ]; then unset EF_LIB_VARIANT; else export EF_LIB_VARIANT=$v; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python tools/prof_image.py > $O/$v.out 2> $O/$v.err || { echo "$v rc=$?"; exit 1; }
  python - $O/$v/run_kernel_stats.csv $v >> $O/summary.txt <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "tm_" in r["Name"]:
        print(sys.argv[2], r["Name"][:40], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us")
PY
done
unset EF_LIB_VARIANT
cat $O/summary.txt
