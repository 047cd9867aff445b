#!/bin/bash
# round-4 batch t (GPU box): rocprof of the current tree with the per-step kernel sequence, and the
# FF1 / dW counter passes refreshed on it (bench.py PMC_TAG)
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
t=r04t
mkdir -p gpurun_out
bash tools/prof_bench.sh $t || exit $?
tail -1 gpurun_out/${t}_bench.log | cut -c1-200
bash tools/pmc_gemm.sh ff1 $t || exit $?
bash tools/pmc_gemm.sh dwtn $t || exit $?
cat gpurun_out/pmc_${t}_ff1.json gpurun_out/pmc_${t}_dwtn.json
