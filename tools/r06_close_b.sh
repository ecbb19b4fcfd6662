#!/bin/bash
# Round-6 closing run, part B: the PMC passes every BENCH traffic figure cites.
# usage: bash tools/r06_close_b.sh <tag> 1|2   (1: C3 scan, C5 screen + bf16 projection;
# 2: C5 fp32 side leg, template localiser + Haar counters, C3 fit breakdown)
cd "$GRAFT_REPO_ROOT" || exit 9
T=${1:-r06/close}
if [ "${2:-1}" = 1 ]; then
  bash tools/r06_capture.sh $T c3 && bash tools/r06_capture.sh $T c5
else
  bash tools/r06_capture.sh $T c5fp32 && bash tools/r06_capture.sh $T image && bash tools/r06_capture.sh $T fit
fi
