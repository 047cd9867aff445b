#!/bin/bash
# round-4 batch p (GPU box): VQ argmax epilogue (max / med3 tracking) -- A/B against HEAD's library
# with bit-equality of the candidates, the VQ / argmax tests, end-to-end A/B
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
t=r04p
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/vq_argmax_ab.py > gpurun_out/${t}_vq_ab.log 2>&1 || { cat gpurun_out/${t}_vq_ab.log; exit 1; }
cat gpurun_out/${t}_vq_ab.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm_tiles.py tests/test_gpu_gemm.py tests/test_gpu_base.py tests/test_gpu_ops.py -k "argmax or vq or VQ" -v -rf --timeout 300 --timeout-method thread > gpurun_out/${t}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/${t}_tests.log | tail -5
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/ab_bench.sh ${t} 3 || exit $?
cat gpurun_out/${t}_ab_bench.log
