#!/bin/bash
# round-5 capture, first call: image PMC, C3 fit breakdown, C5 fp32 side leg PMC
cd "$GRAFT_REPO_ROOT" || exit 9
bash tools/r05_capture.sh ${1:-r05/capA} image && bash tools/r05_capture.sh ${1:-r05/capA} fit && bash tools/r05_capture.sh ${1:-r05/capA} c5fp32
