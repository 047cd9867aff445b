set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_f32path.py tests/test_gpu_model.py tests/test_gpu_mxfp8.py tests/test_gpu_ops.py -x -v -rP --timeout 300 --timeout-method thread > gpurun_out/r03c_f32_tests.log 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_base.py -x -v -rP --timeout 500 --timeout-method thread > gpurun_out/r03c_base_tests.log 2>&1
bash tools/pmc_attn.sh r03c
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r03c_bench.log 2>&1
