#!/bin/bash
# C5 headline (split-bf16 wide scan) for the base library and each variant library
# (tools/wide_variants.sh / tools/variant.sh), alternated twice: value, average launch, frac.
# usage: [SPLIT=3] bash tools/c5_variant_bench.sh <tag> <variant>...   (SPLIT: the scan option, default 1)
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/$1; shift
mkdir -p $O
for rep in 1 2; do
  for v in base "$@"; do
    if [ "$v" = base ]; then unset EF_LIB_VARIANT; else export EF_LIB_VARIANT=$v; fi
    timeout -k 10 240 python bench.py --config c5 --split-opt ${SPLIT:-1} --no-cpu --no-fit --no-image --no-c2 --no-c5 --no-split --steps 10 \
      --repeats 3 > $O/$v.$rep.json 2> $O/$v.$rep.err || exit $?
    python -c "import json; d=json.loads(open('$O/$v.$rep.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['check']['planted_match'])" >> $O/summary.txt
  done
done
echo done
