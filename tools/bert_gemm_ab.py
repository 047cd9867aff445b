"""BERT-base text-tower GEMM shapes (1,024 tokens = batch 8 x 128) through this library's GEMM
(kernels.linear / matmul_nn / matmul_tn, as BertLayerFn calls them) against hipBLASLt
(torch.matmul / addmm on the same bf16 operands), isolated, back to back.
usage (GPU): python tools/bert_gemm_ab.py"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'ctpa-clip_amd'))
import torch  # noqa: E402

from ctclip_mi355x import kernels as K  # noqa: E402

M = 1024


def timeit(fn, n=200):
    for _ in range(10):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


def main():
    torch.manual_seed(0)
    r = lambda *s: (torch.rand(*s, device='cuda') * 2 - 1).bfloat16()  # noqa: E731
    x768, x3072 = r(M, 768), r(M, 3072)
    wqkv, wo, wi, wout = r(2304, 768), r(768, 768), r(3072, 768), r(768, 3072)
    bqkv, bo, bi, bout = (torch.randn(n, device='cuda') for n in (2304, 768, 3072, 768))
    res = torch.randn(M, 768, device='cuda')
    hpre = torch.empty(M, 3072, device='cuda', dtype=torch.bfloat16)
    dy768, dy3072, dy2304 = r(M, 768), r(M, 3072), r(M, 2304)
    cases = [
        ('fwd QKV  1024x2304x768 +bias', lambda: K.linear(x768, wqkv, bias=bqkv),
         lambda: torch.addmm(bqkv.bfloat16(), x768, wqkv.t()), 2 * M * 2304 * 768),
        ('fwd QKV  +bias, split weight', lambda: K.linear(x768, wqkv, bias=bqkv, w_lo=wqkv), None, 4 * M * 2304 * 768),
        ('fwd O    1024x768x768 +b+res32', lambda: K.linear(x768, wo, bias=bo, residual=res, out_dtype=torch.float32),
         lambda: torch.addmm(bo.bfloat16(), x768, wo.t()), 2 * M * 768 * 768),
        ('fwd FF1  1024x3072x768 +b+gelu', lambda: K.linear(x768, wi, bias=bi, act=K.ACT_GELU, out2=hpre),
         lambda: torch.addmm(bi.bfloat16(), x768, wi.t()), 2 * M * 3072 * 768),
        ('fwd FF2  1024x768x3072 +b+res32', lambda: K.linear(x3072, wout, bias=bout, residual=res,
                                                               out_dtype=torch.float32),
         lambda: torch.addmm(bout.bfloat16(), x3072, wout.t()), 2 * M * 768 * 3072),
        ('dX  FF2  1024x3072x768', lambda: K.matmul_nn(dy768, wout), lambda: torch.matmul(dy768, wout),
         2 * M * 3072 * 768),
        ('dX  FF1  1024x768x3072', lambda: K.matmul_nn(dy3072, wi), lambda: torch.matmul(dy3072, wi),
         2 * M * 768 * 3072),
        ('dX  QKV  1024x768x2304', lambda: K.matmul_nn(dy2304, wqkv), lambda: torch.matmul(dy2304, wqkv),
         2 * M * 768 * 2304),
        ('dW  FF1  3072x768 over 1024', lambda: K.matmul_tn(dy3072, x768), lambda: torch.matmul(dy3072.t(), x768),
         2 * M * 768 * 3072),
        ('dW  FF2  768x3072 over 1024', lambda: K.matmul_tn(dy768, x3072), lambda: torch.matmul(dy768.t(), x3072),
         2 * M * 768 * 3072),
        ('dW  QKV  2304x768 over 1024', lambda: K.matmul_tn(dy2304, x768), lambda: torch.matmul(dy2304.t(), x768),
         2 * M * 768 * 2304),
    ]
    tot_k = tot_l = 0.0
    for name, fk, fl, fl_n in cases:
        tk = timeit(fk)
        tl = timeit(fl) if fl else float('nan')
        if fl:
            tot_k += tk
            tot_l += tl
        print(f'{name:34s} ctclip {tk:7.1f} us {fl_n / tk / 1e6:6.1f} TF/s | hipBLASLt {tl:7.1f} us', flush=True)
    print(f'sum of the paired shapes: ctclip {tot_k:.1f} us, hipBLASLt {tot_l:.1f} us', flush=True)


if __name__ == '__main__':
    main()
