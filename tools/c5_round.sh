#!/bin/bash
# Search parity tests, then the C5 bench + PMC passes of the wide kernel.
# usage: bash tools/c5_round.sh <tag>
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_search.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
bash tools/c5_pmc.sh $1
