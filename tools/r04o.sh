#!/bin/bash
# round-4 batch o (GPU box): fold tests (merged q|k l2norm backward, parallel dgamma), the layer /
# model suites, end-to-end A/B of the merged l2norm backward, bench + rocprof
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
t=r04o
mkdir -p gpurun_out
run() {
  local n=$1 to=$2; shift 2
  timeout -k 10 $to python -u -m pytest "$@" -x -v -rf --timeout 300 --timeout-method thread > gpurun_out/${t}_$n.log 2>&1
  local rc=$?
  echo "[$n] rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/${t}_$n.log | tail -6
  return $rc
}
run fold 300 tests/test_gpu_ln1_fold.py || exit $?
run model 900 tests/test_gpu_model.py tests/test_gpu_base.py tests/test_gpu_gemm_ln.py || exit $?
timeout -k 10 600 python -u tools/env_ab.py "" "CTCLIP_QK_BWD_MERGED=0" > gpurun_out/${t}_env_ab.log 2>&1 || exit $?
cat gpurun_out/${t}_env_ab.log
bash tools/prof_bench.sh ${t} || exit $?
tail -1 gpurun_out/${t}_bench.log | cut -c1-200
grep -E "lnfold|l2n_|peg_tile|gemm8p_kernel<true, true, 8>|<true, false, -8>" gpurun_out/${t}_kernel_stats.txt
