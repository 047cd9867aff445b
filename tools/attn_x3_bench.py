"""The split-fp16 x3 attention forward (precise 'split' tower) at the base config (B = 8): spatial
(576 keys, CPB bias, 192 frames) and temporal (24 keys, 4,608 sequences), f32 q / k / v in.
usage: python tools/attn_x3_bench.py   (GPU; CTCLIP_HIP_LIB for A/B)"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'ctpa-clip_amd'))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from ctclip_mi355x import kernels as K  # noqa: E402
from gemm_bench import timeit  # noqa: E402


def main():
    torch.manual_seed(0)
    B, T, Hg, Wg, H, D = 8, 24, 24, 24, 8, 32
    M, hw = B * T * Hg * Wg, Hg * Wg
    q = F.normalize(torch.randn(M, H, D, device='cuda'), dim=-1).reshape(M, H * D)
    kv = torch.randn(M, 2 * H * D, device='cuda')
    kv[:, :H * D] = F.normalize(kv[:, :H * D].reshape(M, H, D), dim=-1).reshape(M, H * D)
    nb = (2 * Hg - 1) * (2 * Wg - 1)
    bias = torch.randn(H, nb, device='cuda') * 0.5
    for name, L, nseq, seq, bu, grid in [('spatial', hw, B * T, (1, hw, 0, 1), bias, (Hg, Wg)),
                                        ('temporal', T, B * hw, (hw, T * hw, 1, hw), None, (0, 0))]:
        ms = timeit(lambda: K.attn_fwd_x3(q, kv[:, :H * D], kv[:, H * D:], L=L, H=H, D=D, nseq=nseq, scale=8.0,
                                          seq=seq, bias_u=bu, grid=grid))
        print(f'x3 {name:8s} fwd {ms * 1e3:8.1f} us', flush=True)


if __name__ == '__main__':
    main()
