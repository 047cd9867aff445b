# PMC passes over the attention kernels of tools/attn_bench.py: bash tools/pmc_attn.sh
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc_a
i=0
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $ctrs --output-format csv -d gpurun_out/pmc_a/p$i -o p -- python tools/attn_bench.py > gpurun_out/pmc_a/log$i 2>&1
done
for k in attn_fwd_kernel attn_bwd_dq_bias attn_bwd_dkv attn_small_bwd; do echo "== $k"; python tools/pmc_table.py gpurun_out/pmc_a $k; done > gpurun_out/pmc_attn.txt
