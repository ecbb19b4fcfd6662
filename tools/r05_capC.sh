#!/bin/bash
# round-5 capture, third call: the C5 screen and bf16 projection PMC
cd "$GRAFT_REPO_ROOT" || exit 9
bash tools/r05_capture.sh ${1:-r05/capC} c5
