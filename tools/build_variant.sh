#!/bin/bash
# Build the library with extra compile flags on one source (A/B variants):
#   tools/build_variant.sh <tag> <source.hip> "<flags>"  -> ctclip_mi355x/libctclip_hip_<tag>.so
set -e
cd "$(dirname "$0")/../ctpa-clip_amd/csrc"
make -s -j8 >/dev/null
tag=$1; src=$2; flags=$3
base=$(basename $src .hip)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -munsafe-fp-atomics $flags -c $src -o build/${base}_$tag.o
objs=$(ls build/*.o | grep -v "_[a-z0-9]*\.o$" | grep -v "build/${base}.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../ctclip_mi355x/libctclip_hip_$tag.so $objs build/${base}_$tag.o
rm -f build/${base}_$tag.o
