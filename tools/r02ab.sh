# GPU box: FF1 FETCH/WRITE under variants: default, no grouped walk, main loop only, epilogue only
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in "def:" "nogrp:CTCLIP_GEMM_GROUP_GX=99" "mainonly:CTCLIP_G256_DEBUG=1" "epionly:CTCLIP_G256_DEBUG=2"; do
  tag=${v%%:*}; e=${v#*:}
  d=gpurun_out/pmc_ab_$tag; rm -rf $d; mkdir -p $d
  i=0
  for ctrs in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    env $e timeout -s KILL 90 rocprofv3 --pmc $ctrs --output-format csv -d $d/p$i -o p -- python tools/gemm_one.py ff1 10 > $d/log$i 2>&1
  done
  echo "== $tag ($e)" >> gpurun_out/r02ab_fetch.txt
  python tools/pmc_table.py $d gemm8p_kernel >> gpurun_out/r02ab_fetch.txt
done
