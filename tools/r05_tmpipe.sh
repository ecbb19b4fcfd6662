#!/bin/bash
# Template localiser: software-pipelined pairs (product) vs variant libraries (e.g. tmold =
# the round-4 loop, EF_TM_PIPE=0; tmtN = tail of N MFMAs): image parity tests, the bench
# frame alternated twice (tools/prof_image.py), then phase stamps of the product build.
# usage: bash tools/r05_tmpipe.sh <tag> <variant>...
cd "$GRAFT_REPO_ROOT" || exit 9
TAG=${1:-r05/tmpipe}; shift
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_image.py -x -v --timeout 120 --timeout-method thread > $O/pytest_image.txt 2>&1 || { echo "pytest rc=$?"; tail -20 $O/pytest_image.txt; exit 1; }
tail -1 $O/pytest_image.txt
for rep in 1 2; do
  for v in product "$@"; do
    if [ $v = product ]; then unset EF_LIB_VARIANT; else export EF_LIB_VARIANT=$v; fi
    timeout -k 10 200 python tools/prof_image.py > $O/$v.$rep.json 2> $O/$v.$rep.err || { echo "$v rc=$?"; exit 1; }
    python -c "import json; d=json.load(open('$O/$v.$rep.json')); t=d['tmatch']; print('$v', t['ms_per_frame_device'], t['frac'])" >> $O/ab.txt
  done
done
unset EF_LIB_VARIANT
cat $O/ab.txt
if [ -f face-detection-recognization-pca_amd/eigenface/_lib/libeigenface_tmstamp.so ]; then
  bash tools/r05_tmstamp.sh $TAG/stamp tmstamp
fi
