#!/bin/bash
# C5 bench for each lib variant: bash tools/wide_sweep.sh <tag> base i1 a1 ...
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/$1; shift
mkdir -p $O
for v in "$@"; do
  if [ "$v" = base ]; then unset EF_LIB_VARIANT; else export EF_LIB_VARIANT=$v; fi
  case $v in a*|*a[0-9]*) export EF_SEARCH_ABL=0;; *) unset EF_SEARCH_ABL;; esac  # ablations: skip the host-key check
  timeout -k 10 200 python bench.py --config c5 --steps 4 --warmup 1 --no-cpu --no-fit > $O/$v.json 2> $O/$v.err || exit $?
  python -c "import json,sys; d=json.loads(open('$O/$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['check'])"
done
