#!/bin/bash
# SYRK DMA-stagger A/B (EF_SYRK_STAGGER variants built by tools/variant.sh): the C3 fit
# (tools/prof_fit.py) with each library, alternated twice: fit seconds and the SYRK's
# hipEvent time.  usage: bash tools/syrk_stagger_ab.sh <tag> <variant>...
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/$1; shift
mkdir -p $O
for rep in ${REPS:-1 2}; do
  for v in base "$@"; do
    if [ "$v" = base ]; then unset EF_LIB_VARIANT; else export EF_LIB_VARIANT=$v; fi
    timeout -k 10 200 python tools/prof_fit.py > $O/$v.$rep.txt 2>&1 || exit $?
    python - "$O/$v.$rep.txt" "$v" >> $O/summary.txt <<'PY'
import ast, sys
line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
d = ast.literal_eval(line)
r = d.get("roofline", {})
print(sys.argv[2], "fit_s", d["gpu_fit_s"], "fit_tr_s", d["gpu_fit_transform_s"], "syrk_ms", r.get("syrk_ms"),
      "syrk_frac", r.get("frac"), "iters", d["eigensolver_iters"], "top3", d["explained_variance_top3"])
PY
  done
done
echo done
