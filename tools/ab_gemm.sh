#!/bin/bash
# Same-box A/B of the GEMM shapes between two library builds, interleaved twice.
#   bash tools/ab_gemm.sh <tag> [libA] [libB]   (default: working tree vs libctclip_hip_old.so)
#   -> gpurun_out/<tag>_ab_gemm.log
set -e
tag=${1:-ab}
d=$PWD/ctpa-clip_amd/ctclip_mi355x
a=${2:-$d/libctclip_hip.so}
b=${3:-$d/libctclip_hip_old.so}
out=gpurun_out/${tag}_ab_gemm.log
mkdir -p gpurun_out; : > $out
for rep in 1 2; do
  for lib in $a $b; do
    echo "== $(basename $lib) ($rep)" >> $out
    CTCLIP_HIP_LIB=$lib GEMM_VARIANTS=8 NO_LIB=1 timeout -k 10 150 python -u tools/gemm_bench.py >> $out 2>&1
  done
done
