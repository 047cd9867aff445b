set -e
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py tests/test_gpu_gemm_tiles.py > gpurun_out/r02p_tests.log 2>&1
: > gpurun_out/r02p_ab.log
for v in 1 0 1 0; do
  echo "== CTCLIP_GEMM_DB=$v" >> gpurun_out/r02p_ab.log
  CTCLIP_GEMM_DB=$v GEMM_VARIANTS=8 NO_LIB=1 timeout -k 10 150 python -u tools/gemm_bench.py >> gpurun_out/r02p_ab.log 2>&1
done
