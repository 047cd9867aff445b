set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k peg -x -q --timeout 120 --timeout-method thread > gpurun_out/r02aa_tests.log 2>&1
bash tools/ab_op_env.sh r02aa peg CTCLIP_PEG_XCD=0 CTCLIP_PEG_XCD=1
