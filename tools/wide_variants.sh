#!/bin/bash
# Build diagnostic / candidate variants of the wide search kernel as
# eigenface/_lib/libeigenface_<tag>.so (selected at run time by EF_LIB_VARIANT=<tag>).
# usage (CPU side): bash tools/wide_variants.sh "i1:-DEF_WIDE_INTERLEAVE=1" "a1:-DEF_WIDE_ABL=1" ...
set -e
cd "$(dirname "$0")/../face-detection-recognization-pca_amd"
make -s
for spec in "$@"; do
  tag=${spec%%:*}; flags=${spec#*:}
  mkdir -p build/v_$tag
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall $flags -c csrc/ef_search_wide.hip -o build/v_$tag/ef_search_wide.o
  objs=$(ls build/*.o | grep -v ef_search_wide.o)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs build/v_$tag/ef_search_wide.o -o eigenface/_lib/libeigenface_$tag.so -ldl
  echo built $tag
done
