set -e
cd $GRAFT_REPO_ROOT
out=gpurun_out/r02x_attn_variants.log; : > $out
d=$PWD/ctpa-clip_amd/ctclip_mi355x
for v in "" nobins nodqa noat; do
  echo "== ${v:-tree}" >> $out
  CTCLIP_HIP_LIB=$d/libctclip_hip${v:+_$v}.so timeout -k 10 120 python -u tools/attn_bench.py 2>&1 | grep "spatial  bwd" >> $out
done
