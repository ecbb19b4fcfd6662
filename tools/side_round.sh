#!/bin/bash
# The side captures of tools/final_round.sh without the GPU suite / headline capture
# (tools/gpu_round.sh): C3 fit trace, C5 capture, image-side trace.  usage: bash tools/side_round.sh <tag>
cd "$GRAFT_REPO_ROOT" || exit 9
bash tools/fit_round.sh $1_fit || exit $?
bash tools/c5_pmc.sh $1_c5 || exit $?
bash tools/img_round.sh $1_img || exit $?
