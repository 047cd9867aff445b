#!/bin/bash
# GPU box: LayerNorm-fused GEMM tests, then same-box A/B of CTCLIP_LN_FUSED on bench.py
set -e
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm_ln.py -x -v -rP --timeout 120 --timeout-method thread \
  > gpurun_out/r03n_ln_tests.log 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_gemm_tiles.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r03n_model_tests.log 2>&1
bash tools/ab_env_bench.sh r03n_lnfused "CTCLIP_LN_FUSED=1" "CTCLIP_LN_FUSED=0"
