#!/bin/bash
# round-4 batch v (GPU box): PEG conv kernels with the two-deep register pipeline (planes two steps
# ahead, residual rows in alternating sets): PEG / fold / model tests, PEG op timing vs HEAD's
# library, end-to-end A/B
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
t=r04v
d=$PWD/ctpa-clip_amd/ctclip_mi355x
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_ln1_fold.py tests/test_gpu_model.py -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/${t}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/${t}_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
out=gpurun_out/${t}_peg_op_ab.log; : > $out
for rep in 1 2 3; do
  for lib in libctclip_hip.so libctclip_hip_old.so; do
    echo "== $lib $rep" >> $out
    CTCLIP_HIP_LIB=$d/$lib OP_ONLY=peg timeout -k 10 150 python -u tools/op_bench.py >> $out 2>&1 || exit $?
  done
done
cat $out
bash tools/ab_bench.sh ${t} 3 || exit $?
cat gpurun_out/${t}_ab_bench.log
