set -e
cd $GRAFT_REPO_ROOT
d=$PWD/ctpa-clip_amd/ctclip_mi355x
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm_tiles.py tests/test_gpu_gemm.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r02az_tests.log 2>&1
bash tools/ab_gemm.sh r02az $d/libctclip_hip.so $d/libctclip_hip_pre0.so
