#!/bin/bash
# Headline bench (no CPU / fit / image legs) for the base library and each variant, alternated
# twice.  usage: bash tools/variant_bench.sh <tag> <variant>...
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/$1; shift
mkdir -p $O
for rep in 1 2; do
  for v in base "$@"; do
    if [ "$v" = base ]; then unset EF_LIB_VARIANT; else export EF_LIB_VARIANT=$v; fi
    timeout -k 10 200 python bench.py --no-cpu --no-fit --no-image --no-c2 --no-c5 > $O/$v.$rep.json 2> $O/$v.$rep.err || exit $?
    python -c "import json; d=json.loads(open('$O/$v.$rep.json').read().strip().splitlines()[-1]); s=d['scan_split_bf16']; print('$v', d['value'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], s['value'], s['roofline']['avg_launch_ms'], s['keys_identical_to_headline'])" >> $O/summary.txt
  done
done
echo done
