#!/bin/bash
# round-4 batch aa (GPU box): the spatial layers' CPB-table gradient accumulated in one buffer
# (no autograd adds on the auxiliary stream): model / base / ops / fold tests, bench + rocprof
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
t=r04aa
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_base.py tests/test_gpu_ops.py tests/test_gpu_ln1_fold.py tests/test_torch_ops.py -x -q -rf --timeout 600 --timeout-method thread > gpurun_out/${t}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/${t}_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/prof_bench.sh $t || exit $?
tail -1 gpurun_out/${t}_bench.log | cut -c1-160
sed -n '/^stream 1/,/top kernels on stream 1/p' gpurun_out/${t}_timeline.txt
tail -14 gpurun_out/${t}_seq.txt
