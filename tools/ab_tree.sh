#!/bin/bash
# same-box A/B of the bench step: this tree vs an older tree checked out (and built) under _ab_old/
# (git worktree, not committed), interleaved runs.  usage: bash tools/ab_tree.sh <tag> [runs]
cd "${GRAFT_REPO_ROOT:-.}"
t=${1:-ab}
n=${2:-3}
for i in $(seq 1 $n); do
  for tree in new old; do
    if [ $tree = new ]; then b=bench.py; else b=_ab_old/bench.py; fi
    timeout -k 10 300 python -u $b --steps 10 --warmup 3 --no-cpu-baseline --no-precise > gpurun_out/${t}_${tree}_$i.log 2>&1 || exit $?
    python - "$tree" gpurun_out/${t}_${tree}_$i.log <<'PY'
import json, sys
l = [x for x in open(sys.argv[2]) if x.startswith('{')][-1]
d = json.loads(l)
print(f"{sys.argv[1]}: {d['value']:.2f} pairs/s  {d['ms_per_step']:.3f} ms/step  vit_fwd {d.get('vit_forward', {}).get('ms')}", flush=True)
PY
  done
done
