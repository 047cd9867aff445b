#!/bin/bash
# GPU box: rocprofv3 kernel-trace summaries of the default bench step for this tree and the older tree
# under _ab_old/ (tools/ab_tree.sh), same box, back to back.   bash tools/prof_tree.sh <tag>
set -e
tag=${1:-run}
export TMPDIR=/tmp
for tree in new old; do
  if [ $tree = new ]; then b=bench.py; x=--no-eval-forward; else b=_ab_old/bench.py; x=; fi
  rm -rf gpurun_out/prof_${tag}_${tree}
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag}_${tree} -o run --output-format rocpd -- \
    python3 -u $b --steps 5 --warmup 2 --no-cpu-baseline --no-precise $x > gpurun_out/${tag}_${tree}_prof_bench.log 2>&1
  db=$(find gpurun_out/prof_${tag}_${tree} -name '*.db' | head -1)
  python tools/rocprof_summary.py "$db" 7 > gpurun_out/${tag}_${tree}_kernel_stats.txt
  rm -rf gpurun_out/prof_${tag}_${tree}
done
