#!/bin/bash
# round-4 batch s (GPU box): the K-step-1 prefetch restricted to the VQ / GEGLU-backward / NN dX
# GEMMs: GEMM + layer tests, per-shape A/B (CTCLIP_GEMM_PRE1 off / on), end to end vs HEAD's library
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
t=r04s
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm_tiles.py tests/test_gpu_gemm.py tests/test_gpu_gemm_ln.py tests/test_gpu_ln1_fold.py tests/test_gpu_model.py -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/${t}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/${t}_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
out=gpurun_out/${t}_gemm_ab.log; : > $out
only="FF1,VQ,Q ,KV,dX  NN        110592x512x2816,dX  NN        110592x1408x512,fused"
for rep in 1 2; do
  for cfg in "CTCLIP_GEMM_PRE1=0" "CTCLIP_GEMM_PRE1=1"; do
    echo "== $cfg ($rep)" >> $out
    env $cfg GEMM_VARIANTS=8 NO_LIB=1 GEMM_ONLY="$only" timeout -k 10 150 python -u tools/gemm_bench.py >> $out 2>&1 || exit $?
  done
done
cat $out
bash tools/ab_bench.sh ${t} 3 || exit $?
cat gpurun_out/${t}_ab_bench.log
