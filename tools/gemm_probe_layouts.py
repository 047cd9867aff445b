"""Main-loop rate of the 8-phase GEMM per operand layout: 4096 x 4096 output (256 tiles, one
per CU), K = 8192 / 16384, f32 output.  NT = both operands K-contiguous (forward), NN = dX
(B MN-contiguous), TN = dW (both MN-contiguous, the split-K weight-gradient layout).
Run with CTCLIP_G256_DEBUG=1 as well to drop the epilogue.   usage: python tools/gemm_probe_layouts.py (GPU)"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'ctpa-clip_amd'))
import torch  # noqa: E402

from ctclip_mi355x import kernels as K  # noqa: E402
from gemm_bench import timeit  # noqa: E402

torch.manual_seed(0)
MN = 4096
r = lambda *s: (torch.rand(*s, device='cuda') * 2 - 1).bfloat16()  # noqa: E731
for Kd in (8192, 16384):
    a_kc, b_kc = r(MN, Kd), r(MN, Kd)          # [M, K], [N, K]
    a_mn, b_mn = r(Kd, MN), r(Kd, MN)          # [K, M], [K, N]
    out = torch.empty(MN, MN, device='cuda')
    fl = 2 * MN * MN * Kd
    cases = [
        ('NT', lambda: K.gemm_raw(MN, MN, Kd, a_kc, Kd, True, b_kc, Kd, True, out, MN)),
        ('NN', lambda: K.gemm_raw(MN, MN, Kd, a_kc, Kd, True, b_mn, MN, False, out, MN)),
        ('TN', lambda: K.gemm_raw(MN, MN, Kd, a_mn, MN, False, b_mn, MN, False, out, MN)),
        ('TT', lambda: K.gemm_raw(MN, MN, Kd, a_mn, MN, False, b_kc, Kd, True, out, MN)),
    ]
    print(f'K={Kd}: ' + ' | '.join(f'{n} {fl / timeit(f, n=10) / 1e9:7.1f} TF/s' for n, f in cases), flush=True)
