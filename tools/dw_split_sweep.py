"""Split-K sweep of the 3D-ViT's small-output weight-gradient GEMMs (dW = dy^T x over the 110,592
tokens of B = 8): Q (256 x 512), attention out (512 x 256), KV (512 x 512), FF2 (512 x 1408).
Times matmul_tn (slab GEMM + slab reduction) per split factor.   usage: python tools/dw_split_sweep.py (GPU)"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'ctpa-clip_amd'))
import torch  # noqa: E402

from ctclip_mi355x import kernels as K  # noqa: E402
from gemm_bench import timeit  # noqa: E402

M = 110592


def main():
    torch.manual_seed(0)
    r = lambda *s: (torch.rand(*s, device='cuda') * 2 - 1).bfloat16()  # noqa: E731
    x512, x256, x1408 = r(M, 512), r(M, 256), r(M, 1408)
    cases = [('dW Q   256x512 ', x512[:, :256], x512), ('dW out 512x256 ', x512, x256),
             ('dW KV  512x512 ', x512, x512), ('dW FF2 512x1408', x512, x1408)]
    for name, dy, x in cases:
        N, Kd = dy.shape[1], x.shape[1]
        flops = 2.0 * M * N * Kd
        row = []
        for s in (16, 24, 32, 48, 64, 96, 128, 192):
            t256 = ((N + 255) // 256) * ((Kd + 255) // 256)
            if t256 * s > 1024 or M // s < 512:
                continue
            ms = timeit(lambda: K.matmul_tn(dy, x, split_k=s))
            row.append(f's{s} {ms * 1e3:6.1f}us {flops / ms / 1e9:6.0f}TF')
        auto = timeit(lambda: K.matmul_tn(dy, x))
        print(f'{name} auto {auto * 1e3:6.1f}us | ' + ' | '.join(row), flush=True)


if __name__ == '__main__':
    main()
