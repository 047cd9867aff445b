set -e
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/r02o_tests.log 2>&1
bash tools/ab_env.sh r02o CTCLIP_DEFER_REDUCE=1 CTCLIP_DEFER_REDUCE=0 2
