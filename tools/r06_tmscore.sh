#!/bin/bash
# Template localiser score blocks: per-map block count (~2048 positions per block, product)
# vs 64 blocks per map (tmscore64 = the previous tree), and the diagnostic build at other
# block sizes (EF_TM_SCORE_POS).  usage: bash tools/r06_tmscore.sh <tag>
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${1:-r06/tmscore}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_image.py -x -q --timeout 120 --timeout-method thread > $O/pytest_image.txt 2>&1 || { echo "pytest rc=$?"; tail -20 $O/pytest_image.txt; exit 1; }
tail -1 $O/pytest_image.txt
run() {  # label, variant lib ('' = product), score_pos
  if [ -n "$2" ]; then export EF_LIB_VARIANT=$2; else unset EF_LIB_VARIANT; fi
  if [ -n "$3" ]; then export EF_TM_SCORE_POS=$3; else unset EF_TM_SCORE_POS; fi
  timeout -k 10 200 python tools/prof_image.py > $O/$1.json 2> $O/$1.err || { echo "$1 rc=$?"; exit 1; }
  python -c "import json; t=json.load(open('$O/$1.json'))['tmatch']; print('$1', t['ms_per_frame_device'], t['frac'])" >> $O/ab.txt
}
for rep in 1 2; do
  run product.$rep "" ""
  run tmscore64.$rep tmscore64 ""
  run pos1024.$rep diag 1024
  run pos4096.$rep diag 4096
done
cat $O/ab.txt
