#!/bin/bash
# GPU box: rocprofv3 kernel summaries of bench.py under two environments (same box, back to back).
#   bash tools/prof_env2.sh <tag> "<VAR=a ...>" "<VAR=b ...>"  -> gpurun_out/<tag>_{a,b}_kernel_stats.txt
set -e
tag=$1
export TMPDIR=/tmp
for side in a b; do
  [ $side = a ] && e=$2 || e=$3
  rm -rf gpurun_out/prof_${tag}_$side
  for kv in $e; do export "$kv"; done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag}_$side -o run --output-format rocpd -- \
    python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-precise --no-eval-forward > gpurun_out/${tag}_${side}_prof_bench.log 2>&1
  for kv in $e; do unset "${kv%%=*}"; done
  db=$(find gpurun_out/prof_${tag}_$side -name '*.db' | head -1)
  { echo "env: $e"; python tools/rocprof_summary.py "$db" 7; } > gpurun_out/${tag}_${side}_kernel_stats.txt
  rm -rf gpurun_out/prof_${tag}_$side
done
