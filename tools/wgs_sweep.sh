#!/bin/bash
# Workgroup-count sweep of the search plan (diagnostic library, EF_SEARCH_WGS) on the
# headline step: fp32 scan and the split side leg.  usage: bash tools/wgs_sweep.sh <tag> <wgs>...
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/$1; shift
mkdir -p $O
export EF_LIB_VARIANT=diag
for w in "$@"; do
  EF_SEARCH_WGS=$w timeout -k 10 200 python bench.py --no-cpu --no-fit --no-image --no-c2 --no-c5 --gallery ${GALLERY:-1000000} > $O/w$w.json 2> $O/w$w.err || exit $?
  python -c "import json; d=json.loads(open('$O/w$w.json').read().strip().splitlines()[-1]); s=d['scan_split_bf16']; print('$w', d['value'], d['roofline']['avg_launch_ms'], s['value'], s['roofline']['avg_launch_ms'], s['keys_identical_to_headline'])" >> $O/summary.txt
done
echo done
