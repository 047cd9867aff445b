# GPU box: full GPU tests, smoke, bench + rocprof summaries (r02v3), FF1 / dW PMC passes (r02c)
set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02z_pytest.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r02z_smoke.log 2>&1
bash tools/prof_bench.sh r02v3
timeout -k 10 400 bash tools/pmc_gemm.sh ff1 r02c
timeout -k 10 400 bash tools/pmc_gemm.sh dwtn r02c
