#!/bin/bash
# Staged resize (ef_image.hip resize_staged_kernel) vs the gather kernel
# (libeigenface_rzgather.so, EF_RESIZE_STAGED=0): the image / Haar / JPEG GPU tests, then
# the image bench's ingest line alternated twice.
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${1:-r05/rzab}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_image.py tests/test_gpu_haar.py > $O/pytest.txt 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for rep in 1 2; do
  for v in product rzgather; do
    if [ $v = product ]; then unset EF_LIB_VARIANT; else export EF_LIB_VARIANT=$v; fi
    timeout -k 10 200 python tools/prof_image.py > $O/$v.$rep.json 2> $O/$v.$rep.err || { echo "$v rc=$?"; tail $O/$v.$rep.err; exit 1; }
    python -c "import json; d=json.load(open('$O/$v.$rep.json')); i=d['ingest']; print('$v', i['ms_per_batch_device'], i['frac'], 'haar', d['haar']['ms_per_frame_device'], 'tm', d['tmatch']['ms_per_frame_device'])" >> $O/ab.txt
  done
done
cat $O/ab.txt
