#!/bin/bash
# Same-box A/B at B = 16 (configs[3]'s per-GPU batch): bench.py with the MX-fp8 image tower vs the
# default bf16 / fp16-operand tower, interleaved.   bash tools/fp8_b16_ab.sh <tag> [reps]
set -e
tag=${1:-fp8}; reps=${2:-2}
out=gpurun_out/${tag}_fp8_b16_ab.log
: > $out
for r in $(seq $reps); do
  for f in "" "--fp8"; do
    v=$(timeout -k 10 300 python -u bench.py --batch 16 --steps 8 --warmup 3 --no-cpu-baseline --no-precise \
          --no-eval-forward $f 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['dtype'])")
    echo "B16 ${f:-bf16} $r $v" >> $out
  done
done
