# PMC passes (one counter group per rocprofv3 run) over any tool script, summarised per kernel:
#   bash tools/pmc_any.sh <tag> "<python script + args>" "<kernel substrings>"
set -e
tag=$1; cmd=$2; kernels=$3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc_$tag
i=0
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $ctrs --output-format csv -d gpurun_out/pmc_$tag/p$i -o p -- python $cmd > gpurun_out/pmc_$tag/log$i 2>&1
done
for k in $kernels; do echo "== $k"; python tools/pmc_table.py gpurun_out/pmc_$tag $k; done > gpurun_out/pmc_$tag.txt
