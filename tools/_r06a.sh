#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/r06
O=gpurun_out/r06/proj2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_project.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.txt 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
B="bench.py --config c5 --steps 5 --warmup 2 --no-cpu --no-fit --no-split --no-image"
for v in wk128 wk64 wide; do
  case $v in wk128) E="EF_PROJ_WK=128";; wk64) E="EF_PROJ_WK=64";; wide) E="EF_PROJ_FRAG=0";; esac
  env EF_LIB_VARIANT=diag $E timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$v -o run -- python $B > $O/t_$v.txt 2>&1 || { echo "trace rc=$?"; tail $O/t_$v.txt; exit 1; }
  python - $O/trace_$v/run_kernel_stats.csv $v <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'project_bf16' in r['Name']: print(sys.argv[2], r['Name'][:60], r['Calls'], r['AverageNs'])
PY
done
P="project_bf16_frag"
timeout -s KILL 180 rocprofv3 --kernel-include-regex "$P" --pmc TCC_EA0_RDREQ_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d $O/proj_req -o run -- python $B > $O/qr.txt 2>&1 || exit $?
python tools/pmc_kernels.py $O/proj_req/run_counter_collection.csv > $O/req.txt; cat $O/req.txt
bash tools/r06_c2proj.sh r06/c2 && bash tools/r06_fit_gap.sh r06/fitgap2
