# GPU box: attention tests (fused backward), then attention timing fused vs two-pass
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k attention -x -v --timeout 120 --timeout-method thread > gpurun_out/r02w_tests.log 2>&1
out=gpurun_out/r02w_attn_ab.log; : > $out
for rep in 1 2; do for e in 0 1; do
  echo "== CTCLIP_ATTN_FUSED=$e ($rep)" >> $out
  CTCLIP_ATTN_FUSED=$e timeout -k 10 120 python -u tools/attn_bench.py >> $out 2>&1
done; done
