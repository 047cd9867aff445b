# PMC passes (one counter group per rocprofv3 run) over one GEMM shape of the step, summarised to
# JSON per launch (tools/pmc_gemm_json.py):
#   bash tools/pmc_gemm.sh <shape> <tag> [lib]     shape: ff1 ff1plain ff2 dxnn dwtn
#   -> gpurun_out/pmc_<tag>_<shape>.json
set -e
which=${1:-ff1}; tag=${2:-r}; lib=${3:-}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
d=gpurun_out/pmc_${tag}_${which}
rm -rf $d; mkdir -p $d
[ -n "$lib" ] && export CTCLIP_HIP_LIB=$lib
i=0
for ctrs in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctrs --output-format csv -d $d/p$i -o p -- python tools/gemm_one.py $which 10 > $d/log$i 2>&1
done
python tools/pmc_gemm_json.py $d gemm8p_kernel > gpurun_out/pmc_${tag}_${which}.json
