cd $GRAFT_REPO_ROOT
set -e
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_ops.py -k "peg" > gpurun_out/r03h_tests.log 2>&1
bash tools/ab_op_env.sh r03h_pegxcd "peg" CTCLIP_PEG_XCD=0 CTCLIP_PEG_XCD=1
bash tools/ab_gemm_env.sh r03h_dyn "" CTCLIP_GEMM_DYN=0 CTCLIP_GEMM_DYN=1
bash tools/ab_env_bench.sh r03h_pegxcd CTCLIP_PEG_XCD=0 CTCLIP_PEG_XCD=1 > gpurun_out/r03h_pegxcd_summary.log 2>&1
