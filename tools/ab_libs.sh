#!/bin/bash
# Same-box GEMM timing across library variants, interleaved:
#   bash tools/ab_libs.sh <tag> "<GEMM_ONLY filter>" <lib tag>...   (lib tag "" = libctclip_hip.so)
set -e
tag=$1; only=$2; shift 2
d=$PWD/ctpa-clip_amd/ctclip_mi355x
out=gpurun_out/${tag}_ab_libs.log
mkdir -p gpurun_out; : > $out
for rep in 1 2; do
  for v in "$@"; do
    lib=$d/libctclip_hip${v:+_$v}.so
    echo "== ${v:-tree} ($rep)" >> $out
    CTCLIP_HIP_LIB=$lib GEMM_VARIANTS=8 NO_LIB=1 GEMM_ONLY="$only" timeout -k 10 150 python -u tools/gemm_bench.py >> $out 2>&1
  done
done
