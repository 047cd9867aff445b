"""Does desynchronising the CUs' epilogue bursts pay?  The persistent 8-phase GEMM delays part of its
first dispatch round (ctclip_gemm_set_stagger: v < 1000 -> every other workgroup of an XCD starts
v x ~2k cycles late; v >= 1000 -> four groups at 0..3 x (v - 1000) units).  Times the K <= 512 /
epilogue-heavy shapes of the step at several staggers, interleaved rounds in one process.
usage: python tools/stagger_sweep.py   (GPU)"""
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'ctpa-clip_amd'))
import torch  # noqa: E402

from ctclip_mi355x import kernels as K, _lib  # noqa: E402

M = 110592


def timeit(fn, n=10):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


def main():
    torch.manual_seed(0)
    r = lambda *s: (torch.rand(*s, device='cuda') * 2 - 1).bfloat16()  # noqa: E731
    x512, x1408, dh = r(M, 512), r(M, 1408), r(M, 2816)
    w1, w2 = r(2816, 512), r(512, 1408)
    g = torch.empty(M, 1408, device='cuda', dtype=torch.bfloat16)
    res = torch.randn(M, 512, device='cuda')
    xo = torch.empty(M, 512, device='cuda', dtype=torch.bfloat16)
    cases = {
        'FF1+GEGLU': lambda: K.linear(x512, w1, act=K.ACT_GEGLU, out2=g),
        'FF1 plain': lambda: K.linear(x512, w1, out=dh),
        'GEGLU-bwd': lambda: K.matmul_nn_geglu_bwd(x512, w2, dh),
        'FF2+res+C2': lambda: K.linear(x1408, w2, residual=res, out_dtype=torch.float32, out2=xo),
        'dX K=2816': lambda: K.matmul_nn(dh, w1),
    }
    vals = [0, 2, 4, 8, 12, 16, 1004, 1006, 1008]
    L = _lib.lib()
    res_ms = {(c, v): [] for c in cases for v in vals}
    for rnd in range(3):
        for v in vals:
            L.ctclip_gemm_set_stagger(v)
            for c, fn in cases.items():
                res_ms[(c, v)].append(timeit(fn))
    L.ctclip_gemm_set_stagger(-1)
    print('median ms over 3 interleaved rounds; stagger units ~2k cycles (>= 1000: 4 groups)')
    print('%-12s' % 'case' + ''.join('%9d' % v for v in vals))
    for c in cases:
        print('%-12s' % c + ''.join('%9.4f' % statistics.median(res_ms[(c, v)]) for v in vals), flush=True)


if __name__ == '__main__':
    main()
