#!/bin/bash
# Round-end capture: full GPU suite + headline bench + C3 trace/PMC (gpu_round.sh), then
# the C5 capture, the C3 fit trace and the image-side trace.  usage: bash tools/final_round.sh <tag>
cd "$GRAFT_REPO_ROOT" || exit 9
bash tools/gpu_round.sh $1 || exit $?
bash tools/c5_pmc.sh $1_c5 || exit $?
bash tools/fit_round.sh $1_fit || exit $?
bash tools/img_round.sh $1_img || exit $?
