# GPU box: full GPU tests, then end-to-end A/B (tree lib vs HEAD lib)
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02s_pytest.log 2>&1
bash tools/ab_bench.sh r02s
