#!/bin/bash
# round-4 batch ab (GPU box): the CPB MLP backward started from the last spatial layer's backward
# right after its attention backward: tests, bench + rocprof, env A/B against the inline CPB
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
t=r04ab
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_base.py tests/test_gpu_ops.py tests/test_torch_ops.py -x -q -rf --timeout 600 --timeout-method thread > gpurun_out/${t}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/${t}_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/prof_bench.sh $t || exit $?
tail -1 gpurun_out/${t}_bench.log | cut -c1-160
sed -n '/^stream 1/,/top kernels on stream 1/p' gpurun_out/${t}_timeline.txt
tail -12 gpurun_out/${t}_seq.txt
timeout -k 10 900 python -u tools/env_ab.py "" "CTCLIP_CPB_AUX=0" > gpurun_out/${t}_env_ab.log 2>&1 || { cat gpurun_out/${t}_env_ab.log; exit 1; }
cat gpurun_out/${t}_env_ab.log
