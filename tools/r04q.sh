#!/bin/bash
# round-4 batch q (GPU box): full GPU suite + smoke + bench + rocprof of the tree after the
# dgamma and VQ-argmax changes (the profile LATEST_ROCPROF points at)
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
t=r04q
bash tools/gpu_round.sh $t || exit $?
head -40 gpurun_out/${t}_kernel_stats.txt
