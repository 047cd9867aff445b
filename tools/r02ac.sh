set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm_tiles.py tests/test_gpu_model.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r02ac_tests.log 2>&1
bash tools/ab_bench.sh r02ac 2
