#!/bin/bash
# round-4 batch aj (GPU box): VQ select with single-code candidates re-scored eight at a time (vs four):
# VQ / base / ops / model tests, in-step vq_select time vs HEAD's library (rocprof), end-to-end A/B
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
t=r04al
d=$PWD/ctpa-clip_amd/ctclip_mi355x
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_base.py tests/test_gpu_ops.py -x -q -rf --timeout 600 --timeout-method thread > gpurun_out/${t}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/${t}_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for v in new old; do
  lib=$d/libctclip_hip.so; [ $v = old ] && lib=$d/libctclip_hip_old.so
  rm -rf gpurun_out/prof_vq_$v
  CTCLIP_HIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_vq_$v -o run --output-format rocpd -- \
    python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-precise > gpurun_out/${t}_$v.log 2>&1 || exit $?
  db=$(find gpurun_out/prof_vq_$v -name '*.db' | head -1)
  python tools/rocprof_summary.py "$db" 7 | grep -E "vq_select|TOTAL" > gpurun_out/${t}_${v}_vq.txt
  rm -rf gpurun_out/prof_vq_$v
  echo "== $v"; cat gpurun_out/${t}_${v}_vq.txt
done
bash tools/ab_bench.sh ${t} 3 || exit $?
cat gpurun_out/${t}_ab_bench.log
