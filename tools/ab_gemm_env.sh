#!/bin/bash
# Same-box GEMM timing across environment settings, interleaved:
#   bash tools/ab_gemm_env.sh <tag> "<GEMM_ONLY filter>" "VAR=a" "VAR=b" ...
set -e
tag=$1; only=$2; shift 2
out=gpurun_out/${tag}_ab_gemm_env.log
mkdir -p gpurun_out; : > $out
for rep in 1 2; do
  for e in "$@"; do
    echo "== $e ($rep)" >> $out
    env $e GEMM_VARIANTS=8 NO_LIB=1 GEMM_ONLY="$only" timeout -k 10 150 python -u tools/gemm_bench.py >> $out 2>&1
  done
done
