set -e
d=$PWD/ctpa-clip_amd/ctclip_mi355x
bash tools/ab_gemm.sh r02g $d/libctclip_hip.so $d/libctclip_hip_sc1.so
bash tools/pmc_gemm.sh ff1 r02g_plain
bash tools/pmc_gemm.sh ff1 r02g_sc1 $d/libctclip_hip_sc1.so
bash tools/pmc_gemm.sh dwtn r02g_plain
CTCLIP_HIP_LIB=$d/libctclip_hip_stamps.so timeout -k 10 120 python -u tools/gemm_stamps.py ff1 ff1plain dx1408 > gpurun_out/r02g_stamps.log 2>&1
