set -e
cd $GRAFT_REPO_ROOT
d=$PWD/ctpa-clip_amd/ctclip_mi355x
CTCLIP_HIP_LIB=$d/libctclip_hip_diag.so timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -k "attn or attention or cpb" --timeout 120 --timeout-method thread > gpurun_out/r02ba_diag_tests.log 2>&1
out=gpurun_out/r02ba_attn_nobin.log; : > $out
for lib in libctclip_hip.so libctclip_hip_nobin.so libctclip_hip_diag.so libctclip_hip.so libctclip_hip_nobin.so libctclip_hip_diag.so; do
  echo "== $lib" >> $out
  CTCLIP_HIP_LIB=$d/$lib timeout -k 10 120 python -u tools/attn_bench.py >> $out 2>&1
done
