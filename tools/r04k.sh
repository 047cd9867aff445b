#!/bin/bash
# round-4 batch k (GPU box): LayerNorm-fold tests (new) + the attention / PEG / l2norm / LN-fused
# layer tests; attention A/B of the arithmetic position table (kb_fast) against HEAD's library;
# end-to-end A/B of the folded LayerNorm (CTCLIP_LN1_FOLD)
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
t=r04k
d=$PWD/ctpa-clip_amd/ctclip_mi355x
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ln1_fold.py tests/test_gpu_ops.py tests/test_gpu_gemm_ln.py -v \
  --timeout 300 --timeout-method thread > gpurun_out/${t}_tests.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "PASS|FAIL|Error|error" gpurun_out/${t}_tests.log | tail -60
if [ $rc -ge 124 ]; then exit $rc; fi
: > gpurun_out/${t}_attn_ab.log
for r in 1 2 3; do
  for lib in libctclip_hip.so libctclip_hip_old.so; do
    echo "== $lib $r" >> gpurun_out/${t}_attn_ab.log
    CTCLIP_HIP_LIB=$d/$lib timeout -k 10 120 python -u tools/attn_bench.py >> gpurun_out/${t}_attn_ab.log 2>&1 || exit $?
  done
done
grep -E "==|spatial" gpurun_out/${t}_attn_ab.log
timeout -k 10 600 python -u tools/env_ab.py "" "CTCLIP_LN1_FOLD=0" > gpurun_out/${t}_env_ab.log 2>&1 || exit $?
cat gpurun_out/${t}_env_ab.log
