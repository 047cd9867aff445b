#!/bin/bash
# round-4 batch d (GPU box): GEMM tile tests (incl. the LDS-relaid epilogue stores, bit-identical),
# extended store probe, epilogue store A/B with staggers.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
t=r04d
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm_tiles.py -v -rP --timeout 300 --timeout-method thread \
  > gpurun_out/${t}_gemm_tests.log 2>&1 || { rc=$?; echo "gemm tests rc=$rc"; tail -20 gpurun_out/${t}_gemm_tests.log; exit $rc; }
tail -2 gpurun_out/${t}_gemm_tests.log
timeout -k 10 120 tools/store_probe > gpurun_out/${t}_store_probe.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/epi_lds_ab.py > gpurun_out/${t}_epi_lds_ab.log 2>&1 || exit $?
cat gpurun_out/${t}_epi_lds_ab.log
