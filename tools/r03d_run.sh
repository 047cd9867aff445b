cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_base.py -v -rP --timeout 500 --timeout-method thread > gpurun_out/r03d_base_tests.log 2>&1
rc=$?; [ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -v -rP --timeout 200 --timeout-method thread -k "attention" > gpurun_out/r03d_attn_tests.log 2>&1
rc=$?; [ $rc -ge 124 ] && exit $rc
set -e
bash tools/ab_env_cmd.sh r03d_attnqb CTCLIP_ATTN_FWD_QB=1 CTCLIP_ATTN_FWD_QB=3 python -u tools/attn_bench.py
bash tools/ab_env_cmd.sh r03d_attnsmax CTCLIP_ATTN_FWD_SMAX=0 CTCLIP_ATTN_FWD_SMAX=1 python -u tools/attn_bench.py
bash tools/ab_env_bench.sh r03d_textfirst CTCLIP_TEXT_FIRST=0 CTCLIP_TEXT_FIRST=1 > gpurun_out/r03d_textfirst_summary.log 2>&1
bash tools/ab_env_bench.sh r03d_textfwdfirst CTCLIP_TEXT_FWD_FIRST=0 CTCLIP_TEXT_FWD_FIRST=1 > gpurun_out/r03d_textfwdfirst_summary.log 2>&1
bash tools/pmc_attn.sh r03d
