"""Isolated timing of the LayerNorm-fused N = 512 GEMMs (ctclip_gemm_ln) against the unfused
GEMM + LayerNorm kernel pairs they replace, at the step's shapes (110,592 tokens)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'ctpa-clip_amd'))
import torch  # noqa: E402

from ctclip_mi355x import kernels as K  # noqa: E402

M = 110592


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
    return s.elapsed_time(e) / n * 1e3


def main():
    torch.manual_seed(0)
    dev = 'cuda'
    o = torch.randn(M, 256, device=dev).bfloat16()
    Wo = (torch.randn(512, 256, device=dev) / 16).bfloat16()
    res = torch.randn(M, 512, device=dev)
    g, b = torch.randn(512, device=dev), torch.randn(512, device=dev)
    x2b = torch.empty(M, 512, device=dev, dtype=torch.bfloat16)

    def fwd_unfused():
        x2f = K.linear(o, Wo, residual=res, out_dtype=torch.float32, out2=x2b)
        K.layernorm_fwd(x2f, g, b, 1e-5)

    def gemm_only():
        K.linear(o, Wo, residual=res, out_dtype=torch.float32, out2=x2b)

    fwd_fused = lambda: K.linear_residual_ln(o, Wo, res, g, b, 1e-5)  # noqa: E731
    xb = torch.randn(M, 512, device=dev).bfloat16()
    _, _, mean, rstd = K.layernorm_fwd(xb.float(), g, b, 1e-5)
    dg = torch.zeros(512, device=dev)
    db = torch.zeros(512, device=dev)
    rows = []
    for name, N in (('LN2 bwd (dh . W1p, K 2816)', 2816), ('LN1 bwd (dq . Wq, K 256)', 256)):
        dy = (torch.randn(M, N, device=dev) * 0.1).bfloat16()
        W = (torch.randn(N, 512, device=dev) / N ** 0.5).bfloat16()

        def unf(dy=dy, W=W):
            d = K.matmul_nn(dy, W)
            K.layernorm_bwd(d, xb, mean, rstd, g, dres=res, dgamma_out=dg, dbeta_out=db)

        def gonly(dy=dy, W=W):
            K.matmul_nn(dy, W)

        def fus(dy=dy, W=W):
            K.matmul_nn_ln_bwd(dy, W, xb, mean, rstd, g, res, dgamma_out=dg, dbeta_out=db)
        rows.append((name, timeit(gonly), timeit(unf), timeit(fus)))
    rows.insert(0, ('LN2 fwd (o . Wo + x1, K 256)', timeit(gemm_only), timeit(fwd_unfused), timeit(fwd_fused)))
    print(f'{"case":34s} {"gemm":>9s} {"gemm+ln":>9s} {"fused":>9s}  (us)')
    for n, a, u, f in rows:
        print(f'{n:34s} {a:9.1f} {u:9.1f} {f:9.1f}')
    print('status', K.ln_fused_status())


if __name__ == '__main__':
    main()
