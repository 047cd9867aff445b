set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03b_gpu_tests.log 2>&1
bash tools/ab_env_bench.sh r03b_textsplit CTCLIP_TEXT_SPLIT=1 CTCLIP_TEXT_SPLIT=0 >> gpurun_out/r03b_ab_summary.log 2>&1
