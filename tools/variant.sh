#!/bin/bash
# Build a variant library eigenface/_lib/libeigenface_<tag>.so with extra flags on ONE source
# (selected at run time with EF_LIB_VARIANT=<tag>).  usage: bash tools/variant.sh <tag> <src.hip> "<flags>"
set -e
cd "$(dirname "$0")/../face-detection-recognization-pca_amd"
make -s
tag=$1; src=$2; flags=$3
base=$(basename $src .hip)
mkdir -p build/v_$tag
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall $flags -c csrc/$src -o build/v_$tag/$base.o
objs=$(ls build/*.o | grep -v "/$base.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs build/v_$tag/$base.o -o eigenface/_lib/libeigenface_$tag.so -ldl
echo built $tag
