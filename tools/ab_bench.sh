#!/bin/bash
# Same-box end-to-end A/B: bench.py with the working-tree library vs libctclip_hip_old.so
# (tools/ab_build.sh <ref>), interleaved.   bash tools/ab_bench.sh <tag> [reps]
set -e
tag=${1:-ab}; reps=${2:-2}
d=$PWD/ctpa-clip_amd/ctclip_mi355x
out=gpurun_out/${tag}_ab_bench.log
: > $out
for r in $(seq $reps); do
  for lib in libctclip_hip.so libctclip_hip_old.so; do
    v=$(CTCLIP_HIP_LIB=$d/$lib timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")
    echo "$lib $r $v" >> $out
  done
done
