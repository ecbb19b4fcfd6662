#!/bin/bash
# SYRK A/B of diagnostic-build switches read once per process (EF_SYRK_NOBAR, EF_SYRK_NB3,
# ...): the C3 fit (tools/prof_fit.py) per setting in its own process, alternated; fit
# seconds, the SYRK's hipEvent time and the top eigenvalues (identical: the integer SYRK
# is exact).  usage: bash tools/syrk_env_ab.sh <tag> VAR=VAL ...   ("base": no switch)
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/$1; shift
mkdir -p $O
export EF_LIB_VARIANT=diag
for rep in ${REPS:-1 2}; do
  for v in base "$@"; do
    if [ "$v" = base ]; then
      timeout -k 10 200 python tools/prof_fit.py > $O/$v.$rep.txt 2>&1 || exit $?
    else
      timeout -k 10 200 env "$v" python tools/prof_fit.py > $O/$v.$rep.txt 2>&1 || exit $?
    fi
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
