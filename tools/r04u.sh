#!/bin/bash
# round-4 batch u (GPU box): q/k l2norm backward with the next row prefetched + no zero-filled grads
# for the bf16 companion outputs: fold / model tests, end-to-end A/B of the library vs HEAD's, rocprof
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
t=r04u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ln1_fold.py tests/test_gpu_model.py tests/test_gpu_base.py -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/${t}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/${t}_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/ab_bench.sh ${t} 3 || exit $?
cat gpurun_out/${t}_ab_bench.log
bash tools/prof_bench.sh $t || exit $?
grep -E "l2n_qk|FillFunctor" gpurun_out/${t}_kernel_stats.txt
