cd $GRAFT_REPO_ROOT
set -e
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_gemm.py -k "dynamic or large_tile" > gpurun_out/r03g_tests.log 2>&1
bash tools/ab_env_bench.sh r03g_dyn CTCLIP_GEMM_DYN=0 CTCLIP_GEMM_DYN=1 > gpurun_out/r03g_dyn_summary.log 2>&1
