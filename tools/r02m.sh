set -e
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "attention" > gpurun_out/r02m_tests.log 2>&1
: > gpurun_out/r02m_attn.log
for v in 1 0 1 0; do
  echo "== CTCLIP_ATTN_DKV_PERSIST=$v" >> gpurun_out/r02m_attn.log
  CTCLIP_ATTN_DKV_PERSIST=$v timeout -k 10 100 python -u tools/attn_bench.py >> gpurun_out/r02m_attn.log 2>&1
done
