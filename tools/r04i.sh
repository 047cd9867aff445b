#!/bin/bash
# round-4 batch i (GPU box): GEMM + attention tests; direct-sc1 epilogue stores (A/B + FF1 counters);
# GEMM variant A/B; what the GELU's erf costs; bench A/B of the sc1 stores
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
t=r04i
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm_tiles.py tests/test_gpu_ops.py -k "not peg and not vq" -v --timeout 300 \
  --timeout-method thread > gpurun_out/${t}_tests.log 2>&1 || { rc=$?; echo "tests rc=$rc"; tail -20 gpurun_out/${t}_tests.log; exit $rc; }
tail -1 gpurun_out/${t}_tests.log
timeout -k 10 300 python -u tools/epi_lds_ab.py > gpurun_out/${t}_epi_lds_ab.log 2>&1 || exit $?
tail -7 gpurun_out/${t}_epi_lds_ab.log
CTCLIP_EPI_LDS=3 bash tools/pmc_gemm.sh ff1 ${t}sc1 || exit $?
python -c "import json; d=json.load(open('gpurun_out/pmc_${t}sc1_ff1.json')); print({k: d[k] for k in ('duration_us_profiled','fetch_bytes_per_launch','write_bytes_per_launch','mfma_busy','l2_hit_rate')})"
timeout -k 10 300 python -u tools/variant_ab.py > gpurun_out/${t}_variant_ab.log 2>&1 || exit $?
tail -8 gpurun_out/${t}_variant_ab.log
timeout -k 10 300 python -u tools/gelu_cost_ab.py > gpurun_out/${t}_gelu_cost_ab.log 2>&1 || exit $?
cat gpurun_out/${t}_gelu_cost_ab.log
timeout -k 10 500 python -u tools/env_ab.py "" "CTCLIP_EPI_LDS=3" > gpurun_out/${t}_env_ab.log 2>&1 || exit $?
cat gpurun_out/${t}_env_ab.log
