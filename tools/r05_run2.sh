set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/r05/c5roles gpurun_out/r05/c5size
SPLIT=3 timeout -k 10 600 bash tools/c5_variant_bench.sh r05/c5roles roles roles4 roles6 || exit $?
for g in 125000 250000; do
  timeout -k 10 200 python bench.py --config c5 --split-opt 3 --gallery $g --no-cpu --no-fit --no-image --no-c2 --no-c5 --no-split --steps 10 --repeats 3 > gpurun_out/r05/c5size/g$g.json 2> gpurun_out/r05/c5size/g$g.err || exit $?
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r05/pytest_gpu_2.txt 2>&1
