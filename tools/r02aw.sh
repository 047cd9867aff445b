set -e
cd $GRAFT_REPO_ROOT
d=$PWD/ctpa-clip_amd/ctclip_mi355x
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm_tiles.py tests/test_gpu_base.py tests/test_gpu_ops.py tests/test_gpu_model.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r02aw_tests.log 2>&1
bash tools/ab_gemm.sh r02aw $d/libctclip_hip.so $d/libctclip_hip_nopl.so
bash tools/ab_bench.sh r02aw 2
