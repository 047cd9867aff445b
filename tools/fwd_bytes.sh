#!/bin/bash
# Per-kernel HBM traffic of the 3D-ViT forward (one train step at B = 8): two rocprofv3 PMC passes
# (FETCH_SIZE, WRITE_SIZE) over tools/fwd_bytes.py, summarised by tools/fwd_bytes_table.py.
#   bash tools/fwd_bytes.sh <tag>  -> gpurun_out/<tag>_fwd_bytes.txt
set -e
tag=${1:-fb}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
d=gpurun_out/pmc_fb_$tag
rm -rf $d; mkdir -p $d
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $d/$c -o p -- python tools/fwd_bytes.py > $d/log_$c 2>&1
done
python tools/fwd_bytes_table.py $d > gpurun_out/${tag}_fwd_bytes.txt
rm -rf $d
