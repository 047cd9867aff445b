"""Time the GEGLU-backward GEMM (the step's FF2 dX + GEGLU backward shape, h in fp16 as the fp16 forward
stores it) on the library CTCLIP_HIP_LIB names.   usage: python tools/geglu_bwd_ab.py   (GPU)"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'ctpa-clip_amd'))
import torch  # noqa: E402

from ctclip_mi355x import kernels as K  # noqa: E402
from gemm_bench import timeit  # noqa: E402


def main():
    torch.manual_seed(0)
    M = 110592
    dy = (torch.randn(M, 512, device='cuda') * 0.1).bfloat16()
    w2 = (torch.randn(512, 1408, device='cuda') * 0.05).bfloat16()
    h = torch.randn(M, 2816, device='cuda').half()
    ms = timeit(lambda: K.matmul_nn_geglu_bwd(dy, w2, h))
    print(f'geglu bwd (h fp16) {ms * 1e3:8.1f} us', flush=True)


if __name__ == '__main__':
    main()
