set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm_tiles.py tests/test_gpu_base.py tests/test_gpu_ops.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r02av_tests.log 2>&1
bash tools/ab_gemm.sh r02av
