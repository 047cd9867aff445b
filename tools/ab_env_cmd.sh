#!/bin/bash
# GPU box: same-box A/B of an environment switch on any command (alternating, 2 rounds each).
#   bash tools/ab_env_cmd.sh <tag> "<ENV=a>" "<ENV=b>" <command...>   -> gpurun_out/<tag>_ab.log
set -e
cd "${GRAFT_REPO_ROOT:-.}"
tag=$1; ea=$2; eb=$3; shift 3
out=gpurun_out/${tag}_ab.log
: > $out
for r in 1 2; do
  for e in "$ea" "$eb"; do
    echo "== $e round $r" >> $out
    env $e timeout -k 10 300 "$@" >> $out 2>&1
  done
done
