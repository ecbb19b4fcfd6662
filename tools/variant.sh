#!/bin/bash
# Build a variant library eigenface/_lib/libeigenface_<tag>.so with extra flags on one source, or
# on several given as a comma-separated list (selected at run time with EF_LIB_VARIANT=<tag>).
# usage: bash tools/variant.sh <tag> <src.hip>[,<src.hip>...] "<flags>"
set -e
cd "$(dirname "$0")/../face-detection-recognization-pca_amd"
make -s
tag=$1; srcs=$2; flags=$3
mkdir -p build/v_$tag
objs=$(ls build/*.o)
for src in ${srcs//,/ }; do
  base=$(basename $src .hip)
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall $flags -c csrc/$src -o build/v_$tag/$base.o
  objs=$(echo "$objs" | grep -v "^build/$base\.o$")
  objs="$objs"$'\n'"build/v_$tag/$base.o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,--no-undefined $objs -o eigenface/_lib/libeigenface_$tag.so -ldl
echo built $tag
