# PMC passes over the attention kernels of tools/attn_bench.py (one counter group per run):
#   bash tools/pmc_attn.sh <tag>  -> gpurun_out/pmc_attn_<tag>.txt
set -e
tag=${1:-a}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
d=gpurun_out/pmc_a_$tag
rm -rf $d; mkdir -p $d
i=0
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VMEM" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_TRANS_F32" ; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv -d $d/p$i -o p -- python tools/attn_bench.py > $d/log$i 2>&1
done
for k in "attn_fwd_kernel<32, true" attn_bwd_dq_bias_dma attn_bwd_dkv_dma attn_small_bwd attn_small_fwd; do echo "== $k"; python tools/pmc_table.py $d "$k"; done > gpurun_out/pmc_attn_$tag.txt
