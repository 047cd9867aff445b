#!/bin/bash
# Same-box op timing (tools/op_bench.py) across environment settings, interleaved:
#   bash tools/ab_op_env.sh <tag> "<OP_ONLY filter>" "VAR=a" "VAR=b" ...
set -e
tag=$1; only=$2; shift 2
out=gpurun_out/${tag}_ab_op_env.log
mkdir -p gpurun_out; : > $out
for rep in 1 2; do
  for e in "$@"; do
    echo "== $e ($rep)" >> $out
    env $e OP_ONLY="$only" timeout -k 10 150 python -u tools/op_bench.py >> $out 2>&1
  done
done
