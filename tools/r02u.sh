# GPU box: VQ/argmax + tile tests, VQ GEMM timing tree vs HEAD, end-to-end A/B
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm_tiles.py tests/test_gpu_gemm.py tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r02u_tests.log 2>&1
bash tools/ab_libs.sh r02u "VQ,FF1,dX  NN+res" "" old
bash tools/ab_bench.sh r02u
