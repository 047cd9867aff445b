"""hipBLASLt (torch.matmul) on the contrastive step's GEMM shapes, for comparison with
tools/gemm_bench.py.  Not part of the product path.   usage: python tools/blas_ref.py   (GPU)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402

from gemm_bench import timeit, M  # noqa: E402


def main():
    torch.manual_seed(0)
    r = lambda *s: (torch.rand(*s, device='cuda') * 2 - 1).bfloat16()  # noqa: E731
    shapes = [('FF1 NT', M, 2816, 512), ('FF2 NT', M, 512, 1408), ('Q   NT', M, 256, 512), ('KV  NT', M, 512, 512),
              ('dX  NN', M, 512, 2816), ('dX  NN', M, 1408, 512)]
    for name, m, n, k in shapes:
        a, w = r(m, k), r(n, k)
        ms = timeit(lambda: torch.matmul(a, w.t()))
        print(f'{name} {m}x{n}x{k}  hipblaslt {ms:7.3f} ms {2 * m * n * k / ms / 1e9:7.1f} TF/s', flush=True)
    for name, m, n, k in [('dW  TN', 2816, 512, M), ('dW  TN', 512, 512, M)]:
        a, b = r(k, m), r(k, n)
        ms = timeit(lambda: torch.matmul(a.t(), b))
        print(f'{name} {m}x{n}x{k}  hipblaslt {ms:7.3f} ms {2 * m * n * k / ms / 1e9:7.1f} TF/s', flush=True)


if __name__ == '__main__':
    main()
