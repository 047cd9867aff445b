set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k peg -x -q --timeout 120 --timeout-method thread > gpurun_out/r02v_tests.log 2>&1
CTCLIP_PEG_FIXED=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k peg -x -q --timeout 120 --timeout-method thread >> gpurun_out/r02v_tests.log 2>&1
bash tools/ab_op_env.sh r02v peg CTCLIP_PEG_FIXED=0 CTCLIP_PEG_FIXED=1
