set -e
cd $GRAFT_REPO_ROOT
d=$PWD/ctpa-clip_amd/ctclip_mi355x
CTCLIP_HIP_LIB=$d/libctclip_hip_stamps.so timeout -k 10 120 python -u tools/gemm_stamps.py ff1 geglubwd dx1408 dwq > gpurun_out/r02aj_stamps.log 2>&1
bash tools/pmc_gemm.sh geglubwd r02aj
bash tools/pmc_gemm.sh dx1408 r02aj
bash tools/pmc_gemm.sh dwq r02aj
