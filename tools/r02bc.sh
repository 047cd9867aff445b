set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r02bc_gpu_tests.log 2>&1
out=gpurun_out/r02bc_attn_ws_ab.log; : > $out
for e in 1 0 1 0; do
  echo "== CTCLIP_ATTN_BIAS_WS=$e" >> $out
  CTCLIP_ATTN_BIAS_WS=$e timeout -k 10 120 python -u tools/attn_bench.py >> $out 2>&1
done
bash tools/ab_env.sh r02bc "CTCLIP_ATTN_BIAS_WS=1" "CTCLIP_ATTN_BIAS_WS=0" 2
