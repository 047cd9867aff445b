#!/bin/bash
# round-4 batch ai (GPU box, diagnostic): in-step cost of the VQ select's full-group f32 re-score --
# rocprof of the bench with the library and with a build that treats every group as single
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
d=$PWD/ctpa-clip_amd/ctclip_mi355x
for v in base diag; do
  lib=$d/libctclip_hip.so; [ $v = diag ] && lib=$d/libctclip_hip_diag.so
  rm -rf gpurun_out/prof_vq_$v
  CTCLIP_HIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_vq_$v -o run --output-format rocpd -- \
    python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-precise > gpurun_out/r04ai_$v.log 2>&1 || exit $?
  db=$(find gpurun_out/prof_vq_$v -name '*.db' | head -1)
  python tools/rocprof_summary.py "$db" 7 | grep -E "vq_select|TOTAL" > gpurun_out/r04ai_${v}_vq.txt
  rm -rf gpurun_out/prof_vq_$v
  echo "== $v"; cat gpurun_out/r04ai_${v}_vq.txt
done
