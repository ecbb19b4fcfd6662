#!/bin/bash
# round-5 capture, second call: the default bench line and the C3 scan PMC
cd "$GRAFT_REPO_ROOT" || exit 9
bash tools/r05_capture.sh ${1:-r05/capB} bench && bash tools/r05_capture.sh ${1:-r05/capB} c3
