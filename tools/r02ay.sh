set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 > gpurun_out/r02ay_gpus2_gloo.log 2>&1
timeout -k 10 300 python -u bench.py --batch 16 --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/r02ay_bf16_b16.log 2>&1
timeout -k 10 300 python -u bench.py --fp8 --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/r02ay_fp8_b16.log 2>&1
