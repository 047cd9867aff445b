#!/bin/bash
# round-4 measurement batch b (GPU box): f32-tower kernel profile, store-burst probe, fp8 vs bf16 at
# B = 16, refreshed GEMM counters, the f32-path tests.  Any step that fails stops the script.
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
t=r04b
timeout -k 10 300 python -u -m pytest tests/test_gpu_f32path.py -v -rP --timeout 300 --timeout-method thread \
  > gpurun_out/${t}_f32_tests.log 2>&1 || { rc=$?; echo "f32 tests rc=$rc"; [ $rc -lt 124 ] || exit $rc; }
timeout -k 10 120 tools/store_probe > gpurun_out/${t}_store_probe.log 2>&1
echo "store probe ok"
rm -rf gpurun_out/prof_${t}
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${t} -o run --output-format rocpd -- \
  python3 -u bench.py --f32-tower --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${t}_f32_prof_bench.log 2>&1
db=$(find gpurun_out/prof_${t} -name '*.db' | head -1)
python tools/rocprof_summary.py "$db" 4 > gpurun_out/${t}_f32_kernel_stats.txt
rm -rf gpurun_out/prof_${t}
echo "f32 profile ok"
timeout -k 10 300 python -u bench.py --fp8 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/${t}_bench_fp8_b16.log 2>&1
timeout -k 10 300 python -u bench.py --batch 16 --steps 10 --warmup 3 --no-cpu-baseline --no-precise > gpurun_out/${t}_bench_bf16_b16.log 2>&1
echo "b16 benches ok"
bash tools/pmc_gemm.sh ff1 ${t}
bash tools/pmc_gemm.sh dwtn ${t}
echo "pmc ok"
