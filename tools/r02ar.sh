set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_dropout.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r02ar_tests.log 2>&1
for e in "CTCLIP_QKV_WGRAD=1 CTCLIP_LNB_WIDE=1" "CTCLIP_QKV_WGRAD=0 CTCLIP_LNB_WIDE=0"; do
  echo "== $e" >> gpurun_out/r02ar_tower.log
  env $e timeout -k 10 240 python -u tools/tower_alone.py >> gpurun_out/r02ar_tower.log 2>&1
done
bash tools/ab_env.sh r02ar "CTCLIP_QKV_WGRAD=1 CTCLIP_LNB_WIDE=1" "CTCLIP_QKV_WGRAD=0 CTCLIP_LNB_WIDE=0" 3
