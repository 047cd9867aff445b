set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_base.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r02ad_tests.log 2>&1
timeout -k 10 300 python -u tools/op_census.py > gpurun_out/r02ad_op_census.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r02ad_bench.log 2>&1
