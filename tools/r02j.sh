set -e
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py tests/test_gpu_gemm_tiles.py > gpurun_out/r02j_tests.log 2>&1
bash tools/ab_gemm.sh r02j
