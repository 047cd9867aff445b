set -e
cd $GRAFT_REPO_ROOT
out=gpurun_out/r02be_lnb_cap.log; : > $out
for c in 1024 2048 4096 1024 2048 4096; do
  echo "== CTCLIP_LNB_CAP=$c" >> $out
  CTCLIP_LNB_CAP=$c OP_ONLY=ln_bwd timeout -k 10 120 python -u tools/op_bench.py >> $out 2>&1
done
bash tools/ab_env.sh r02be "CTCLIP_LNB_CAP=2048" "CTCLIP_LNB_CAP=1024" 2
