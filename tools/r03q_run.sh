#!/bin/bash
# GPU box: fused-LN + BERT-fusion tests, then same-box A/B of the switches
set -e
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm_ln.py tests/test_gpu_dropout.py -x -v -rP --timeout 200 \
  --timeout-method thread > gpurun_out/r03q_tests.log 2>&1
bash tools/ab_env_multi.sh r03q "CTCLIP_LN_FUSED=1" "CTCLIP_LN_FUSED=0" "CTCLIP_BERT_FUSE=0" "CTCLIP_BERT_NODROP=1"
