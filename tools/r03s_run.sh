#!/bin/bash
# GPU box: text-tower split-layer precision sweep, then same-box A/B of the split-layer count
set -e
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/bert_split_sweep.py > gpurun_out/r03s_split_sweep.log 2>&1
bash tools/ab_env_multi.sh r03s "CTCLIP_TEXT_SPLIT_LAYERS=12" "CTCLIP_TEXT_SPLIT_LAYERS=4" "CTCLIP_TEXT_SPLIT_LAYERS=0"
