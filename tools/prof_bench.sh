#!/bin/bash
# GPU box: bench + rocprofv3 kernel-trace summary of the same command.
#   bash tools/prof_bench.sh <tag>   -> gpurun_out/<tag>_bench.log, gpurun_out/<tag>_kernel_stats.txt
set -e
tag=${1:-run}
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py > gpurun_out/${tag}_bench.log 2>&1
rm -rf gpurun_out/prof_${tag}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag} -o run --output-format rocpd -- \
  python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-precise --no-eval-forward > gpurun_out/${tag}_prof_bench.log 2>&1
db=$(find gpurun_out/prof_${tag} -name '*.db' | head -1)
python tools/rocprof_summary.py "$db" 7 > gpurun_out/${tag}_kernel_stats.txt
python tools/rocprof_grid.py "$db" "" 7 > gpurun_out/${tag}_grid_stats.txt
python tools/rocprof_streams.py "$db" 200 > gpurun_out/${tag}_streams.txt || true
python tools/rocprof_timeline.py "$db" > gpurun_out/${tag}_timeline.txt || true
python tools/rocprof_seq.py "$db" > gpurun_out/${tag}_seq.txt || true
python tools/rocprof_copies.py "$db" 7 > gpurun_out/${tag}_copies.txt || true
rm -rf gpurun_out/prof_${tag}
