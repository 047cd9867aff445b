#!/bin/bash
# round-4 batch h (GPU box): GEMM tile tests (LDS-relaid epilogue incl. the sc1 form), epilogue store
# A/B (plain / LDS-relaid / LDS-relaid sc1 x stagger), FF1 counters with the sc1 form
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
t=r04h
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm_tiles.py tests/test_torch_ops.py -v --timeout 300 --timeout-method thread \
  > gpurun_out/${t}_gemm_tests.log 2>&1 || { rc=$?; echo "gemm tests rc=$rc"; tail -20 gpurun_out/${t}_gemm_tests.log; exit $rc; }
tail -1 gpurun_out/${t}_gemm_tests.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_f32path.py -k "attention" -v --timeout 120 \
  --timeout-method thread > gpurun_out/${t}_attn_tests.log 2>&1 || { rc=$?; echo "attn tests rc=$rc"; tail -20 gpurun_out/${t}_attn_tests.log; exit $rc; }
tail -1 gpurun_out/${t}_attn_tests.log
timeout -k 10 300 python -u tools/attn_lazy_ab.py > gpurun_out/${t}_attn_lazy_ab.log 2>&1 || exit $?
grep "LAZY=" gpurun_out/${t}_attn_lazy_ab.log
timeout -k 10 400 python -u tools/epi_lds_ab.py > gpurun_out/${t}_epi_lds_ab.log 2>&1 || exit $?
tail -7 gpurun_out/${t}_epi_lds_ab.log
CTCLIP_EPI_LDS=2 bash tools/pmc_gemm.sh ff1 ${t}lds2 || exit $?
python -c "import json; d=json.load(open('gpurun_out/pmc_${t}lds2_ff1.json')); print({k: d[k] for k in ('duration_us_profiled','fetch_bytes_per_launch','write_bytes_per_launch','mfma_busy','l2_hit_rate')})"
timeout -k 10 300 python -u tools/variant_ab.py > gpurun_out/${t}_variant_ab.log 2>&1 || exit $?
tail -8 gpurun_out/${t}_variant_ab.log
