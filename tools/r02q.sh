# GPU box: full GPU test suite, smoke, then bench + rocprof kernel-trace summaries (tag r02v2)
set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02q_pytest.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r02q_smoke.log 2>&1
bash tools/prof_bench.sh r02v2
