set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "layernorm or patch" -x -q --timeout 120 --timeout-method thread > gpurun_out/r02af_tests.log 2>&1
d=$PWD/ctpa-clip_amd/ctclip_mi355x
out=gpurun_out/r02af_ln_ab.log; : > $out
for rep in 1 2; do for lib in libctclip_hip.so libctclip_hip_old.so; do
  echo "== $lib ($rep)" >> $out
  CTCLIP_HIP_LIB=$d/$lib OP_ONLY=ln_ timeout -k 10 120 python -u tools/op_bench.py >> $out 2>&1
done; done
