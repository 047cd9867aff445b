#!/bin/bash
# round-4 batch m (GPU box): end-to-end A/B of the LayerNorm fold; attention A/B of the arithmetic
# position table (kb_fast) against the library before it (438acfa); bench + rocprof of the tree
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
t=r04m
d=$PWD/ctpa-clip_amd/ctclip_mi355x
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/env_ab.py "" "CTCLIP_LN1_FOLD=0" > gpurun_out/${t}_env_ab.log 2>&1 || exit $?
cat gpurun_out/${t}_env_ab.log
: > gpurun_out/${t}_attn_ab.log
for r in 1 2 3; do
  for lib in libctclip_hip.so libctclip_hip_old.so; do
    echo "== $lib $r" >> gpurun_out/${t}_attn_ab.log
    CTCLIP_HIP_LIB=$d/$lib timeout -k 10 120 python -u tools/attn_bench.py >> gpurun_out/${t}_attn_ab.log 2>&1 || exit $?
  done
done
grep -E "==|spatial" gpurun_out/${t}_attn_ab.log
bash tools/prof_bench.sh ${t} || exit $?
tail -1 gpurun_out/${t}_bench.log
head -30 gpurun_out/${t}_kernel_stats.txt
