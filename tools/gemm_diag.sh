#!/bin/bash
# GEMM decomposition on the GPU box: full kernels, main loop only (epilogue skipped), epilogue
# only (main loop skipped), K sweep.   bash tools/gemm_diag.sh <tag>  -> gpurun_out/<tag>_gemm_diag.log
set -e
tag=${1:-diag}
out=gpurun_out/${tag}_gemm_diag.log
mkdir -p gpurun_out
echo "== full (variants ${GEMM_VARIANTS:-8,1})" > $out
NO_LIB=${NO_LIB:-1} timeout -k 10 180 python -u tools/gemm_bench.py >> $out 2>&1
echo "== main loop only (CTCLIP_G256_DEBUG=1)" >> $out
CTCLIP_G256_DEBUG=1 NO_LIB=1 GEMM_VARIANTS=8 timeout -k 10 180 python -u tools/gemm_bench.py >> $out 2>&1
echo "== epilogue + prologue only (CTCLIP_G256_DEBUG=2)" >> $out
CTCLIP_G256_DEBUG=2 NO_LIB=1 GEMM_VARIANTS=8 timeout -k 10 180 python -u tools/gemm_bench.py >> $out 2>&1
echo "== K sweep" >> $out
timeout -k 10 120 python -u tools/gemm_bench.py ksweep >> $out 2>&1
