#!/bin/bash
# round-4 batch g (GPU box): attention tests + lazy-rescale A/B, then the full round (GPU tests,
# smoke, bench, rocprof summary of the bench command)
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
t=r04g
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "attention" -v --timeout 120 --timeout-method thread \
  > gpurun_out/${t}_attn_tests.log 2>&1 || { rc=$?; echo "attn tests rc=$rc"; tail -20 gpurun_out/${t}_attn_tests.log; exit $rc; }
tail -1 gpurun_out/${t}_attn_tests.log
timeout -k 10 300 python -u tools/attn_lazy_ab.py > gpurun_out/${t}_attn_lazy_ab.log 2>&1 || exit $?
cat gpurun_out/${t}_attn_lazy_ab.log
bash tools/gpu_round.sh ${t}
