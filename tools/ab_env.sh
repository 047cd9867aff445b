#!/bin/bash
# Same-box end-to-end A/B of one environment switch: bench.py with "$2" vs "$3" (env assignments),
# interleaved.   bash tools/ab_env.sh <tag> "VAR=1" "VAR=0" [reps]
set -e
tag=$1; a=$2; b=$3; reps=${4:-2}
out=gpurun_out/${tag}_ab_env.log
: > $out
for r in $(seq $reps); do
  for e in "$a" "$b"; do
    v=$(env $e timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")
    echo "$e $r $v" >> $out
  done
done
