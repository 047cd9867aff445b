#!/bin/bash
# GPU box: attention kernels + end-to-end, working-tree library vs libctclip_hip_old.so (tools/ab_build.sh <ref>)
set -e
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
d=$PWD/ctpa-clip_amd/ctclip_mi355x
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_base.py -x -q -k "attention or stages" --timeout 250 --timeout-method thread > gpurun_out/r03w_attn_tests.log 2>&1
: > gpurun_out/r03w_attn_ab.log
for r in 1 2 3; do
  for lib in libctclip_hip.so libctclip_hip_old.so; do
    echo "== $lib $r" >> gpurun_out/r03w_attn_ab.log
    CTCLIP_HIP_LIB=$d/$lib timeout -k 10 120 python -u tools/attn_bench.py >> gpurun_out/r03w_attn_ab.log 2>&1
  done
done
bash tools/ab_bench.sh r03w 2
