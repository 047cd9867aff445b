#!/bin/bash
# GPU box: same-box A/B of an environment switch on bench.py (alternating, 2 rounds each).
#   bash tools/ab_env_bench.sh <tag> "<ENV=a>" "<ENV=b>" [bench args...]
set -e
cd "${GRAFT_REPO_ROOT:-.}"
tag=$1; ea=$2; eb=$3; shift 3
out=gpurun_out/${tag}_ab.log
: > $out
for r in 1 2; do
  for e in "$ea" "$eb"; do
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
        cur = line.split()[1]
    elif line.startswith('{'):
        res.setdefault(cur, []).append(json.loads(line)['value'])
for k, v in res.items():
    print(k, v, 'mean', sum(v) / len(v))
PY
