#!/bin/bash
# round-4 batch e (GPU box): patch-LN strip kernel XCD order A/B, patch tests
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
t=r04e
timeout -k 10 200 python -u -m pytest tests/test_gpu_ops.py -k "patch" -v --timeout 120 --timeout-method thread \
  > gpurun_out/${t}_patch_tests.log 2>&1 || { rc=$?; echo "patch tests rc=$rc"; tail -20 gpurun_out/${t}_patch_tests.log; exit $rc; }
tail -2 gpurun_out/${t}_patch_tests.log
timeout -k 10 300 python -u tools/patch_ab.py > gpurun_out/${t}_patch_ab.log 2>&1 || exit $?
cat gpurun_out/${t}_patch_ab.log
timeout -k 10 400 python -u tools/dw_variant_ab.py > gpurun_out/${t}_dw_variant_ab.log 2>&1 || exit $?
tail -8 gpurun_out/${t}_dw_variant_ab.log
