set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for mode in fp8 bf16; do
  flag=""; [ $mode = fp8 ] && flag="--fp8"
  rm -rf gpurun_out/prof_am_$mode
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_am_$mode -o run --output-format rocpd -- \
    python3 -u bench.py --steps 4 --warmup 2 --batch 16 --no-cpu-baseline $flag > gpurun_out/r02am_${mode}_bench.log 2>&1
  db=$(find gpurun_out/prof_am_$mode -name '*.db' | head -1)
  python tools/rocprof_summary.py "$db" 6 > gpurun_out/r02am_${mode}_kernel_stats.txt
  python tools/rocprof_timeline.py "$db" > gpurun_out/r02am_${mode}_timeline.txt || true
  rm -rf gpurun_out/prof_am_$mode
done
