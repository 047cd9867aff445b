"""Attention kernels at the base config (B = 8: 110,592 tokens, 8 heads x 32): spatial (576 keys,
CPB bias, 192 frames) and temporal (24 keys, 4608 sequences), forward and backward."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'ctpa-clip_amd'))
import torch  # noqa: E402

from ctclip_mi355x import kernels as K  # noqa: E402
from gemm_bench import timeit  # noqa: E402


def main():
    torch.manual_seed(0)
    B, T, Hg, Wg, H, D = 8, 24, 24, 24, 8, 32
    M, hw = B * T * Hg * Wg, Hg * Wg
    r = lambda *s: (torch.randn(*s, device='cuda') * 0.3).bfloat16()  # noqa: E731
    q, k, v, do = r(M, H * D), r(M, H * D), r(M, H * D), r(M, H * D)
    nb = (2 * Hg - 1) * (2 * Wg - 1)
    bias = torch.randn(H, nb, device='cuda') * 0.5
    only = os.environ.get('ATTN_ONLY', '')   # 'spatial' | 'temporal' | '' (both)
    for name, L, nseq, seq, bu, grid in [('spatial', hw, B * T, (1, hw, 0, 1), bias, (Hg, Wg)),
                                        ('temporal', T, B * hw, (hw, T * hw, 1, hw), None, (0, 0))]:
        if only and name != only:
            continue
        o, lse = K.attn_fwd(q, k, v, L=L, H=H, D=D, nseq=nseq, scale=8.0, seq=seq, bias_u=bu, grid=grid)
        fl = 4.0 * nseq * H * L * L * D
        o16 = os.environ.get('O16', '0') != '0'    # also write O's fp16 copy (the fp16 to_out GEMM's A)
        ms = timeit(lambda: K.attn_fwd(q, k, v, L=L, H=H, D=D, nseq=nseq, scale=8.0, seq=seq, bias_u=bu, grid=grid,
                                       want_o16=o16))
        print(f'{name:8s} fwd {ms * 1e3:8.1f} us {fl / ms / 1e9:7.1f} TF/s (fp16 copy {int(o16)})', flush=True)
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        du = torch.zeros_like(bias) if bu is not None else None

        def bwd():
            K.attn_bwd(q, k, v, o, lse, do, dq, dk, dv, L=L, H=H, D=D, nseq=nseq, scale=8.0, seq=seq, bias_u=bu,
                       dbias_u=du, grid=grid)
        ms = timeit(bwd)
        print(f'{name:8s} bwd {ms * 1e3:8.1f} us {2.5 * fl / ms / 1e9:7.1f} TF/s (2.5x fwd flops)', flush=True)


if __name__ == '__main__':
    main()
