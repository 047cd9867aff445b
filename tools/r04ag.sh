#!/bin/bash
# round-4 batch ag (GPU box): FeedForward weights packed on the auxiliary stream at the start of the
# image tower's forward: tests, env A/B
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
t=r04ag
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_base.py tests/test_gpu_f32path.py -x -q -rf --timeout 600 --timeout-method thread > gpurun_out/${t}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/${t}_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python -u tools/env_ab.py "" "CTCLIP_PREPACK_AUX=0" > gpurun_out/${t}_env_ab.log 2>&1 || { cat gpurun_out/${t}_env_ab.log; exit 1; }
cat gpurun_out/${t}_env_ab.log
