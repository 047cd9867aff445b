cd $GRAFT_REPO_ROOT
set -e
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_gemm.py tests/test_gpu_gemm_tiles.py > gpurun_out/r03i_tests.log 2>&1
bash tools/ab_gemm_env.sh r03i_bal "" CTCLIP_GEMM_BALANCE=0 CTCLIP_GEMM_BALANCE=1
bash tools/ab_env_bench.sh r03i_bal CTCLIP_GEMM_BALANCE=0 CTCLIP_GEMM_BALANCE=1 > gpurun_out/r03i_bal_summary.log 2>&1
