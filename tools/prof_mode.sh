#!/bin/bash
# GPU box: rocprofv3 kernel-trace summary of bench.py in one image-tower precision mode (5 + 2 steps).
#   bash tools/prof_mode.sh <tag> <bf16|split|f32>   -> gpurun_out/<tag>_<mode>_kernel_stats.txt (+ _seq)
set -e
tag=${1:-run}
mode=${2:-split}
export TMPDIR=/tmp
rm -rf gpurun_out/prof_${tag}
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag} -o run --output-format rocpd -- \
  python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-precise --no-eval-forward --vit-precision ${mode} \
  > gpurun_out/${tag}_${mode}_prof_bench.log 2>&1
db=$(find gpurun_out/prof_${tag} -name '*.db' | head -1)
python tools/rocprof_summary.py "$db" 7 > gpurun_out/${tag}_${mode}_kernel_stats.txt
python tools/rocprof_seq.py "$db" > gpurun_out/${tag}_${mode}_seq.txt || true
python tools/rocprof_seq.py "$db" all > gpurun_out/${tag}_${mode}_seq_all.txt || true
rm -rf gpurun_out/prof_${tag}
