# GPU box: GEMM tile tests, then the GEMM A/B against HEAD's build
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm_tiles.py tests/test_gpu_gemm.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r02r_tests.log 2>&1
bash tools/ab_gemm.sh r02res2
