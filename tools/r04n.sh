#!/bin/bash
# round-4 batch n (GPU box): full GPU suite + smoke + bench + rocprof of the LN1-fold tree, then the
# attention A/B of the arithmetic position table against the library before it (438acfa)
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
t=r04n
d=$PWD/ctpa-clip_amd/ctclip_mi355x
bash tools/gpu_round.sh $t || exit $?
head -40 gpurun_out/${t}_kernel_stats.txt
: > gpurun_out/${t}_attn_ab.log
for r in 1 2 3; do
  for lib in libctclip_hip.so libctclip_hip_old.so; do
    echo "== $lib $r" >> gpurun_out/${t}_attn_ab.log
    CTCLIP_HIP_LIB=$d/$lib timeout -k 10 120 python -u tools/attn_bench.py >> gpurun_out/${t}_attn_ab.log 2>&1 || exit $?
  done
done
grep -E "==|spatial" gpurun_out/${t}_attn_ab.log
