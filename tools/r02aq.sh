set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
rm -rf gpurun_out/prof_aq
TOWER_ONLY=bert timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_aq -o run --output-format rocpd -- \
  python3 -u tools/tower_alone.py > gpurun_out/r02aq_log.txt 2>&1
db=$(find gpurun_out/prof_aq -name '*.db' | head -1)
python tools/rocprof_summary.py "$db" 8 > gpurun_out/r02aq_bert_kernel_stats.txt
python tools/rocprof_grid.py "$db" "" 8 > gpurun_out/r02aq_bert_grid_stats.txt
rm -rf gpurun_out/prof_aq
