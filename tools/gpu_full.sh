#!/bin/bash
# GPU box: the round-end sequence in one call -- GPU tests, smoke, bench + rocprof summary.
#   bash tools/gpu_full.sh <tag> [pytest -k expr]
#   -> gpurun_out/<tag>_gpu_tests.log, <tag>_smoke.log, <tag>_bench.log, <tag>_kernel_stats.txt ...
set -e
cd "${GRAFT_REPO_ROOT:-.}"
tag=${1:-run}
sel=${2:-}
mkdir -p gpurun_out
if [ -n "$sel" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread -k "$sel" \
    > gpurun_out/${tag}_gpu_tests.log 2>&1
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread \
    > gpurun_out/${tag}_gpu_tests.log 2>&1
fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1
bash tools/prof_bench.sh ${tag}
