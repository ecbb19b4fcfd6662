#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/r06
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_image.py tests/test_gpu_jpeg.py > gpurun_out/r06/pytest_img.txt 2>&1 || { echo "img rc=$?"; tail -30 gpurun_out/r06/pytest_img.txt; exit 1; }
tail -1 gpurun_out/r06/pytest_img.txt
bash tools/r06_proj.sh r06/proj && bash tools/r06_fit_gap.sh r06/fitgap2
