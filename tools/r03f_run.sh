cd $GRAFT_REPO_ROOT
set -e
timeout -k 10 300 python -u tools/tower_alone.py > gpurun_out/r03f_tower_alone.log 2>&1
bash tools/ab_env_bench.sh r03f_gridcap240 CTCLIP_GEMM_GRID_CAP=0 CTCLIP_GEMM_GRID_CAP=240 > gpurun_out/r03f_gridcap240_summary.log 2>&1
bash tools/ab_env_bench.sh r03f_gridcap224 CTCLIP_GEMM_GRID_CAP=0 CTCLIP_GEMM_GRID_CAP=224 > gpurun_out/r03f_gridcap224_summary.log 2>&1
timeout -k 10 300 python -u tools/host_ahead.py 10 > gpurun_out/r03f_host_ahead.log 2>&1
CTCLIP_TEXT_FIRST=0 timeout -k 10 300 python -u tools/host_ahead.py 10 >> gpurun_out/r03f_host_ahead.log 2>&1
