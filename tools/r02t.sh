# GPU box: argmax GEMM epilogue A/B (LDS-staged vs transposed) + tile tests with the TR argmax
set -e
cd $GRAFT_REPO_ROOT
out=gpurun_out/r02t_argmax.log; : > $out
for rep in 1 2; do for e in 0 1; do
  echo "== ARGMAX_TR=$e ($rep)" >> $out
  CTCLIP_GEMM_ARGMAX_TR=$e GEMM_VARIANTS=8 NO_LIB=1 GEMM_ONLY="VQ" timeout -k 10 150 python -u tools/gemm_bench.py >> $out 2>&1
done; done
CTCLIP_GEMM_ARGMAX_TR=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm_tiles.py tests/test_gpu_gemm.py tests/test_gpu_ops.py -k "argmax or vq" -x -q --timeout 120 --timeout-method thread >> $out 2>&1
