"""The forward / dX GEMM shapes of the 3D-ViT step on the three large-tile kernel variants
(ctclip_gemm_set_variant: 8 = 8-phase 256x256x64 persistent, one workgroup per CU; 1 = 128x256x32,
two workgroups per CU -- one's epilogue can run beside the other's main loop; 2 = 256x256x32 4-slot
ring).  The GEGLU backward (act 4) and l2norm (act 5) epilogues exist only in the 8-phase kernel.
Interleaved rounds in one process; median ms.  usage: python tools/variant_ab.py   (GPU)"""
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
    w1, w2, wkv, wo, x256 = r(2816, 512), r(512, 1408), r(512, 512), r(512, 256), r(M, 256)
    g = torch.empty(M, 1408, device='cuda', dtype=torch.bfloat16)
    res = torch.randn(M, 512, device='cuda')
    xo = torch.empty(M, 512, device='cuda', dtype=torch.bfloat16)
    cases = {
        'FF1+GEGLU': lambda: K.linear(x512, w1, act=K.ACT_GEGLU, out2=g),
        'FF2+res+C2': lambda: K.linear(x1408, w2, residual=res, out_dtype=torch.float32, out2=xo),
        'Wo+res+C2': lambda: K.linear(x256, wo, residual=res, out_dtype=torch.float32, out2=xo),
        'KV bf16': lambda: K.linear(x512, wkv),
        'dX K=2816': lambda: K.matmul_nn(dh, w1),
        'dX K=512': lambda: K.matmul_nn(x512, wkv),
    }
    L = _lib.lib()
    vals = (8, 1, 2)
    res_ms = {(c, v): [] for c in cases for v in vals}
    outs = {}
    for rnd in range(3):
        for v in vals:
            L.ctclip_gemm_set_variant(v)
            for c, fn in cases.items():
                res_ms[(c, v)].append(timeit(fn))
                if rnd == 0:
                    o = fn()
                    outs[(c, v)] = o.float().clone()
        print(f'round {rnd} done', flush=True)
    L.ctclip_gemm_set_variant(8)
    for c in cases:
        for v in vals:
            assert torch.equal(outs[(c, v)], outs[(c, 8)]) or \
                (outs[(c, v)] - outs[(c, 8)]).abs().max().item() <= 1e-2 * outs[(c, 8)].abs().max().item(), (c, v)
    print('median ms over 3 interleaved rounds; columns = variant')
    print('%-12s' % 'case' + ''.join('%10d' % v for v in vals))
    for c in cases:
        print('%-12s' % c + ''.join('%10.4f' % statistics.median(res_ms[(c, v)]) for v in vals), flush=True)


if __name__ == '__main__':
    main()
