#!/bin/bash
# JPEG ingest early-upload A/B (one process per setting)
set -o pipefail
mkdir -p gpurun_out/r06
cd "$(dirname "$0")/.."
EF_LIB_VARIANT=diag EF_JPEG_EARLY_UP=0 timeout -k 10 240 python -u tools/r06_jpeg_ab.py > gpurun_out/r06/jpeg_ab_off.json &&
EF_LIB_VARIANT=diag EF_JPEG_EARLY_UP=1 timeout -k 10 240 python -u tools/r06_jpeg_ab.py > gpurun_out/r06/jpeg_ab_on.json &&
timeout -k 10 240 python -u tools/r06_jpeg_ab.py > gpurun_out/r06/jpeg_ab_prod.json &&
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests -k "jpeg" > gpurun_out/r06/jpeg_tests.txt 2>&1
