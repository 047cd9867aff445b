#!/bin/bash
# Same-box end-to-end A/B of two whole trees (Python + library): the working tree vs ./ab_old
# (git archive <ref> | tar -x -C ab_old; build its library in place), interleaved.
#   bash tools/ab_tree.sh <tag> [reps]
set -e
cd "${GRAFT_REPO_ROOT:-.}"
tag=${1:-ab}; reps=${2:-3}
out=gpurun_out/${tag}_ab_tree.log
: > $out
for r in $(seq $reps); do
  for d in . ab_old; do
    v=$(cd $d && timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")
    echo "$d $r $v" | tee -a $out
  done
done
