#!/bin/bash
# round-4 batch c (GPU box): f32-path tests after the PEG / l2norm / patch-LN / attention rewrites,
# the f32-mode kernel profile, the extended store probe, the default bench line.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
t=r04c
timeout -k 10 300 python -u -m pytest tests/test_gpu_f32path.py -v -rP --timeout 300 --timeout-method thread \
  > gpurun_out/${t}_f32_tests.log 2>&1 || { rc=$?; echo "f32 tests rc=$rc"; [ $rc -lt 124 ] || exit $rc; }
tail -2 gpurun_out/${t}_f32_tests.log
timeout -k 10 120 tools/store_probe > gpurun_out/${t}_store_probe.log 2>&1 || exit $?
rm -rf gpurun_out/prof_${t}
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${t} -o run --output-format rocpd -- \
  python3 -u bench.py --f32-tower --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${t}_f32_prof_bench.log 2>&1 || exit $?
db=$(find gpurun_out/prof_${t} -name '*.db' | head -1)
python tools/rocprof_summary.py "$db" 4 > gpurun_out/${t}_f32_kernel_stats.txt
rm -rf gpurun_out/prof_${t}
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/${t}_bench.log 2>&1 || exit $?
tail -1 gpurun_out/${t}_bench.log | cut -c1-400
