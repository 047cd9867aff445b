set -e
cd $GRAFT_REPO_ROOT
d=$PWD/ctpa-clip_amd/ctclip_mi355x
for lib in libctclip_hip_seg2.so libctclip_hip_seg1.so; do
  CTCLIP_HIP_LIB=$d/$lib timeout -k 10 200 python -u -m pytest tests/test_gpu_ops.py -x -q -k peg --timeout 120 --timeout-method thread > gpurun_out/r02at_tests_$lib.log 2>&1
done
out=gpurun_out/r02at_peg_ab.log; : > $out
for rep in 1 2; do
for lib in libctclip_hip.so libctclip_hip_seg2.so libctclip_hip_seg1.so; do
  echo "== $lib" >> $out
  CTCLIP_HIP_LIB=$d/$lib OP_ONLY=peg timeout -k 10 120 python -u tools/op_bench.py >> $out 2>&1
done
done
