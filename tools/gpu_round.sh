#!/bin/bash
# GPU box: GPU tests (not stopping at the first failure), smoke, bench + rocprof summary, then any
# extra command.  A step that ends by a signal, a time limit or a crash (exit status >= 124 other
# than a plain failure) ends the script: no further GPU step runs after it.
#   bash tools/gpu_round.sh <tag> [extra command...]
cd "${GRAFT_REPO_ROOT:-.}"
tag=${1:-run}
shift
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rP --timeout 300 --timeout-method thread \
  > gpurun_out/${tag}_gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/${tag}_gpu_tests.log
if [ $rc -ge 124 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1
rc=$?
echo "smoke rc=$rc"; tail -2 gpurun_out/${tag}_smoke.log
if [ $rc -ge 124 ]; then exit $rc; fi
bash tools/prof_bench.sh ${tag}
rc=$?
echo "prof_bench rc=$rc"; tail -1 gpurun_out/${tag}_bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
if [ $# -gt 0 ]; then
  "$@"
fi
