#!/bin/bash
# Round-3 fit studies on one box: int8 MFMA clock ceiling (tools/micro/bf16_clock i), the
# covariance operand copy A/B (tools/transpose_ab.sh) and the C3 fit capture (tools/fit_round.sh).
# usage: bash tools/r03_fit_ab.sh <tag>
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 120 ./tools/micro/bf16_clock i > $O/i8_clock.json 2> $O/i8_clock.err || exit $?
bash tools/transpose_ab.sh $1_tab || exit $?
bash tools/fit_round.sh $1_fit || exit $?
