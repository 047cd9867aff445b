set -e
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "attention" > gpurun_out/r02i_tests.log 2>&1
echo "== DMA dq kernel" > gpurun_out/r02i_attn.log
timeout -k 10 100 python -u tools/attn_bench.py >> gpurun_out/r02i_attn.log 2>&1
echo "== generic dq kernel" >> gpurun_out/r02i_attn.log
CTCLIP_ATTN_DQ_DMA=0 timeout -k 10 100 python -u tools/attn_bench.py >> gpurun_out/r02i_attn.log 2>&1
echo "== DMA dq kernel" >> gpurun_out/r02i_attn.log
timeout -k 10 100 python -u tools/attn_bench.py >> gpurun_out/r02i_attn.log 2>&1
