#!/bin/bash
# GPU box: same-box bench.py comparison of N environment settings (alternating, 2 rounds each).
#   bash tools/ab_env_multi.sh <tag> "<ENV=a [ENV2=b]>" "<ENV=c>" ... -- [bench args...]
set -e
cd "${GRAFT_REPO_ROOT:-.}"
tag=$1; shift
envs=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do envs+=("$1"); shift; done
[ "$1" == "--" ] && shift
out=gpurun_out/${tag}_ab.log
: > $out
for r in 1 2; do
  for e in "${envs[@]}"; do
    echo "== $e round $r" >> $out
    env $e timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" 2>&1 | grep '^{' >> $out
  done
done
python - "$out" <<'PY'
import json, sys
cur = None
res = {}
for line in open(sys.argv[1]):
    if line.startswith('=='):
        cur = line[3:].rsplit(' round', 1)[0]
    elif line.startswith('{'):
        res.setdefault(cur, []).append(json.loads(line)['value'])
for k, v in res.items():
    print(f'{k:50s}', v, 'mean', round(sum(v) / len(v), 2))
PY
