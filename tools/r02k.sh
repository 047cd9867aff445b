set -e
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_gemm.py tests/test_gpu_gemm_tiles.py tests/test_gpu_model.py > gpurun_out/r02k_tests.log 2>&1
bash tools/prof_bench.sh r02k
