#!/bin/bash
# Template localiser A/B: product (column blocks past the map edge skipped) vs
# libeigenface_tmfull.so (EF_TM_NCB_SKIP=0), alternated twice, then the GPU parity tests.
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${1:-r05/tmab}
mkdir -p $O
for rep in 1 2; do
  for v in product tmfull; do
    if [ $v = product ]; then unset EF_LIB_VARIANT; else export EF_LIB_VARIANT=$v; fi
    timeout -k 10 200 python tools/prof_image.py > $O/$v.$rep.json 2> $O/$v.$rep.err || { echo "$v rc=$?"; exit 1; }
    python -c "import json,sys; d=json.load(open('$O/$v.$rep.json')); t=d['tmatch']; print('$v', t['ms_per_frame_device'], t['frac'])" >> $O/ab.txt
  done
done
unset EF_LIB_VARIANT
cat $O/ab.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread $2 > $O/pytest.txt 2>&1 || { echo "pytest rc=$?"; tail -20 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
