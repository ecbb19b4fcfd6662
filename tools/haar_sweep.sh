#!/bin/bash
# Haar parity tests, then the Haar bench section per (EF_HAAR_SPLIT_FROM, EF_HAAR_SPLITW)
# combination, then a kernel trace of the default.
# usage: bash tools/haar_sweep.sh <tag> [from:waves ...]   (default combos 6:4 6:8 6:16)
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/$1; shift
mkdir -p $O
combos=${@:-"6:4 6:8 6:16"}
timeout -k 10 300 python -u -m pytest tests/test_gpu_haar.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for c in $combos; do
  f=${c%%:*}; w=${c#*:}
  EF_HAAR_SPLIT_FROM=$f EF_HAAR_SPLITW=$w timeout -k 10 200 python tools/prof_image.py > $O/f${f}w$w.json 2>/dev/null || exit $?
  python -c "import json; d=json.load(open('$O/f${f}w$w.json'))['haar']; print('from=$f W=$w', d['frames_per_s'], d['ms_per_frame_device'], d['detections'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ir -o run -- python tools/prof_image.py > $O/out.txt 2>&1 || exit $?
grep -E "haar|Kernel_Name" /tmp/ir/run_kernel_trace.csv > $O/haar_trace.csv
