#!/bin/bash
# Template localiser, product library vs variants (tools/variant.sh), alternated twice:
# tools/tm_micro.py shapes + the bench's 640x480 x 60-map frame.  usage: bash tools/tm_variant_ab.sh <tag> <variant>...
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/$1; shift
mkdir -p $O
for rep in 1 2; do
  for v in base "$@"; do
    if [ "$v" = base ]; then unset EF_LIB_VARIANT; else export EF_LIB_VARIANT=$v; fi
    timeout -k 10 200 python -u tools/tm_micro.py > $O/$v.$rep.micro.txt 2>&1 || exit $?
    timeout -k 10 300 python bench.py --no-cpu --no-fit --no-c2 --no-c5 --no-split --steps 3 --repeats 1 > $O/$v.$rep.json 2> $O/$v.$rep.err || exit $?
    python - "$O" "$v" "$rep" >> $O/summary.txt <<'PY'
import json, sys
o, v, rep = sys.argv[1:4]
d = json.loads(open(f"{o}/{v}.{rep}.json").read().strip().splitlines()[-1])
t = d["tmatch"]
micro = [json.loads(l) for l in open(f"{o}/{v}.{rep}.micro.txt") if l.startswith("{")]
print(v, "tmatch_ms", t["ms_per_frame_device"], "frac", t["frac"], "micro_ms", [m["ms"] for m in micro])
PY
  done
done
echo done
