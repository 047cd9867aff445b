# GPU box: MX-fp8 tests (epilogues + model), then a configs[3] fp8 bench at B=16 and bf16 at B=16
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_mxfp8.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r02y_tests.log 2>&1
timeout -k 10 300 python -u bench.py --fp8 --no-cpu-baseline --steps 6 --warmup 2 > gpurun_out/r02y_bench_fp8_b16.log 2>&1
timeout -k 10 300 python -u bench.py --batch 16 --no-cpu-baseline --steps 6 --warmup 2 > gpurun_out/r02y_bench_bf16_b16.log 2>&1
