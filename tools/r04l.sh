#!/bin/bash
# round-4 batch l (GPU box): the LayerNorm-fold kernels in isolation first, then whole layers, then
# the suites that run the model; stops at the first failing stage
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
t=r04l
mkdir -p gpurun_out
run() {   # name, timeout, pytest args...
  local n=$1 to=$2; shift 2
  timeout -k 10 $to python -u -m pytest "$@" -x -v -rf --timeout 300 --timeout-method thread > gpurun_out/${t}_$n.log 2>&1
  local rc=$?
  echo "[$n] rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/${t}_$n.log | tail -12
  return $rc
}
run kernels 300 tests/test_gpu_ln1_fold.py -k "stats or gemm or wgrad" || exit $?
run layers 300 tests/test_gpu_ln1_fold.py -k "layer" || exit $?
run gemmln 400 tests/test_gpu_gemm_ln.py || exit $?
run model 900 tests/test_gpu_model.py tests/test_gpu_base.py || exit $?
