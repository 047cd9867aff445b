"""Wave-quantisation probe of the persistent 8-phase GEMM: time the step's N = 512 shapes at token
counts whose 256 x 256 tile count is 3, 3.375 (the step: M = 110,592) and 4 rounds of 256 workgroups.
If 3.375 rounds cost as much as 4, the last partial round is the price of the step's tile count.
usage: python tools/quant_probe.py (GPU)"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'ctpa-clip_amd'))
import torch  # noqa: E402

from ctclip_mi355x import kernels as K  # noqa: E402


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


def main():
    torch.manual_seed(0)
    r = lambda *s: (torch.rand(*s, device='cuda') * 2 - 1).bfloat16()  # noqa: E731
    w2, w1 = r(512, 1408), r(2816, 512)
    for M in (98304, 110592, 131072):
        x1408, dh = r(M, 1408), r(M, 2816)
        res = torch.randn(M, 512, device='cuda')
        t_ff2 = timeit(lambda: K.linear(x1408, w2, residual=res, out_dtype=torch.float32))
        t_dx = timeit(lambda: K.matmul_nn(dh, w1))
        tiles = (M // 256) * 2
        print(f'M={M:6d} tiles={tiles:4d} rounds={tiles / 256:5.3f}: FF2+res32 {t_ff2 * 1e3:7.1f} us '
              f'({t_ff2 * 1e3 / (tiles / 256):6.1f} per round-equivalent) | dX K=2816 {t_dx * 1e3:7.1f} us '
              f'({t_dx * 1e3 / (tiles / 256):6.1f})', flush=True)
        del x1408, dh, res


if __name__ == '__main__':
    main()
