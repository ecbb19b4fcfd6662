#!/bin/bash
# Round-6 profile capture (after the kernels are final): the default bench line, its
# kernel trace, and separate PMC passes (FETCH_SIZE / WRITE_SIZE / SQ) for every search
# kernel a BENCH traffic figure cites — the C3 fp32 scan, the C5 bf16 screen, the C5 fp32
# side leg and the C5 bf16 projection — summarised by tools/pmc_summary.py.
# usage: bash tools/r05_capture.sh <tag> [part]   part: bench | c3 | c5 | c5fp32 | image | fit | all (default)
# image: the template localiser's MFMA busy and the Haar stage groups' TA busy
# (tools/img_summary.py); fit: the C3 fit's per-kernel breakdown (tools/fit_breakdown.py).
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 9
TAG=${1:-r06cap}
PART=${2:-all}
O=gpurun_out/$TAG
mkdir -p $O
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  echo "== $name: $*" >> $O/steps.log
  timeout -k 10 $to "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "== $name rc=$rc" >> $O/steps.log
  return $rc
}
pmc3() {  # tag, kernel regex, config, bench args...
  local t=$1 R=$2 cfg=$3; shift 3
  step ${t}_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${t}_trace -o run -- python "$@" || return $?
  step ${t}_fetch 180 rocprofv3 --kernel-include-regex "$R" --pmc FETCH_SIZE --output-format csv -d $O/${t}_fetch -o run -- python "$@" || return $?
  step ${t}_write 180 rocprofv3 --kernel-include-regex "$R" --pmc WRITE_SIZE --output-format csv -d $O/${t}_write -o run -- python "$@" || return $?
  step ${t}_sq 180 rocprofv3 --kernel-include-regex "$R" --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY --output-format csv -d $O/${t}_sq -o run -- python "$@" || return $?
  python tools/pmc_summary.py $O/${t}_fetch/run_counter_collection.csv $O/${t}_write/run_counter_collection.csv \
    $O/${t}_sq/run_counter_collection.csv $O/${t}_trace/run_kernel_stats.csv $O/pmc_summary_$cfg.json $cfg > $O/${t}_summary.txt
}
if [ "$PART" = all ] || [ "$PART" = bench ]; then
  step bench 900 python bench.py || exit $?
fi
if [ "$PART" = all ] || [ "$PART" = c3 ]; then
  pmc3 c3 "search_kernel<128, 0, false, false, 0>" c3 bench.py --steps 5 --warmup 2 --no-cpu --no-fit --no-c2 --no-c5 --no-image || exit $?
fi
if [ "$PART" = all ] || [ "$PART" = c5 ]; then
  pmc3 c5hi "search_wide16" c5hi bench.py --config c5 --split-opt 3 --steps 3 --warmup 1 --no-cpu --no-fit --no-split --no-image || exit $?
  pmc3 c5proj "project_bf16_frag" c5proj bench.py --config c5 --split-opt 3 --steps 3 --warmup 1 --no-cpu --no-fit --no-split --no-image || exit $?
fi
if [ "$PART" = all ] || [ "$PART" = c5fp32 ]; then
  pmc3 c5 "search_wide_kernel<512" c5 bench.py --config c5 --search fp32 --steps 3 --warmup 1 --no-cpu --no-fit --no-split --no-image || exit $?
fi
if [ "$PART" = all ] || [ "$PART" = image ]; then
  R="tm_corr|haar_cascade"
  step img_trace 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/img_trace -o run -- python tools/prof_image.py || exit $?
  step img_sq 180 rocprofv3 --kernel-include-regex "$R" --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT --output-format csv -d $O/img_sq -o run -- python tools/prof_image.py || exit $?
  step img_ta 180 rocprofv3 --kernel-include-regex "$R" --pmc TA_BUSY_avr GRBM_GUI_ACTIVE FETCH_SIZE --output-format csv -d $O/img_ta -o run -- python tools/prof_image.py || exit $?
  python tools/img_summary.py $O/img_sq/run_counter_collection.csv $O/img_ta/run_counter_collection.csv \
    $O/img_trace/run_kernel_stats.csv $O > $O/img_summary.txt || exit $?
fi
if [ "$PART" = all ] || [ "$PART" = fit ]; then
  step fit_trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/fit_trace -o run -- python tools/prof_fit.py || exit $?
  python tools/fit_breakdown.py $O/fit_trace/run_kernel_trace.csv > $O/fit_c3_breakdown.txt || exit $?
fi
echo done >> $O/steps.log
