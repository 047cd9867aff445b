#!/bin/bash
# round-4 batch j (GPU box): attention tests on the working tree; attention forward A/B (lazy-path
# max exchanges skipped) against libctclip_hip_old.so; what the text tower costs inside the step
# (tower_alone) and what its hi / lo split weights cost (env A/B)
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
t=r04j
d=$PWD/ctpa-clip_amd/ctclip_mi355x
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "attention" -v --timeout 250 --timeout-method thread \
  > gpurun_out/${t}_attn_tests.log 2>&1 || { rc=$?; echo "tests rc=$rc"; tail -20 gpurun_out/${t}_attn_tests.log; exit $rc; }
tail -1 gpurun_out/${t}_attn_tests.log
: > gpurun_out/${t}_attn_ab.log
for r in 1 2 3; do
  for lib in libctclip_hip.so libctclip_hip_old.so; do
    echo "== $lib $r" >> gpurun_out/${t}_attn_ab.log
    CTCLIP_HIP_LIB=$d/$lib timeout -k 10 120 python -u tools/attn_bench.py >> gpurun_out/${t}_attn_ab.log 2>&1 || exit $?
  done
done
grep -E "==|fwd" gpurun_out/${t}_attn_ab.log
timeout -k 10 300 python -u tools/tower_alone.py > gpurun_out/${t}_tower_alone.log 2>&1 || exit $?
cat gpurun_out/${t}_tower_alone.log | tail -6
timeout -k 10 500 python -u tools/env_ab.py "" "CTCLIP_TEXT_SPLIT=0" > gpurun_out/${t}_env_ab.log 2>&1 || exit $?
cat gpurun_out/${t}_env_ab.log
