"""Per-shape timing of the MFMA GEMM on the contrastive step's main shapes (B = 8 tokens = 110,592).
usage: python tools/gemm_bench.py   (GPU)"""
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
    return s.elapsed_time(e) / n


def main():
    torch.manual_seed(0)
    r = lambda *s: (torch.rand(*s, device='cuda') * 2 - 1).bfloat16()  # noqa: E731
    x512, x1408 = r(M, 512), r(M, 1408)
    w1, w2, wq, wkv = r(2816, 512), r(512, 1408), r(256, 512), r(512, 512)
    g = torch.empty(M, 1408, device='cuda', dtype=torch.bfloat16)
    res = torch.randn(M, 512, device='cuda')
    x256, wo = r(M, 256), r(512, 256)
    xo = torch.empty(M, 512, device='cuda', dtype=torch.bfloat16)
    cb = r(8192, 512)
    cand = torch.empty(M, 128, 2, device='cuda')
    cand2 = torch.empty(M, 128, device='cuda')
    dh = r(M, 2816)
    x512h, w1h = x512.half(), w1.half()
    sqa, sqb = r(8192, 8192), r(8192, 8192)
    sqo = torch.empty(8192, 8192, device='cuda', dtype=torch.bfloat16)
    cases = [
        ('FF1 NT+GEGLU  110592x2816x512', lambda: K.linear(x512, w1, act=K.ACT_GEGLU, out2=g), 2 * M * 2816 * 512),
        ('FF1 f16 GEGLU 110592x2816x512', lambda: K.linear(x512h, w1h, act=K.ACT_GEGLU, out2=g,
                                                           out_dtype=torch.float16), 2 * M * 2816 * 512),
        ('FF1 NT plain  110592x2816x512', lambda: K.linear(x512, w1, out=dh), 2 * M * 2816 * 512),
        ('FF2 NT+res32  110592x512x1408', lambda: K.linear(x1408, w2, residual=res, out_dtype=torch.float32),
         2 * M * 512 * 1408),
        ('FF2 NT+res32+C2 110592x512x1408', lambda: K.linear(x1408, w2, residual=res, out_dtype=torch.float32,
                                                             out2=xo), 2 * M * 512 * 1408),
        ('Wo  NT+res32+C2 110592x512x256', lambda: K.linear(x256, wo, residual=res, out_dtype=torch.float32,
                                                            out2=xo), 2 * M * 512 * 256),
        ('dX  NN+res32  110592x512x512', lambda: K.matmul_nn(x512, wkv, residual=res, out_dtype=torch.float32),
         2 * M * 512 * 512),
        ('VQ  NT argmax 110592x8192x512', lambda: K.gemm_raw(M, 8192, 512, x512, 512, True, cb, 512, True, cand, 128,
                                                          C2=cand2, ldc2=128, act=K.ACT_ARGMAX), 2 * M * 8192 * 512),
        ('Q   NT        110592x256x512', lambda: K.linear(x512, wq), 2 * M * 256 * 512),
        ('KV  NT        110592x512x512', lambda: K.linear(x512, wkv), 2 * M * 512 * 512),
        ('dX  NN        110592x512x2816', lambda: K.matmul_nn(dh, w1), 2 * M * 512 * 2816),
        ('dX  NN        110592x1408x512', lambda: K.matmul_nn(x512, w2), 2 * M * 1408 * 512),
        ('dG+geglu_bwd  fused', lambda: K.matmul_nn_geglu_bwd(x512, w2, dh), 2 * M * 1408 * 512),
        ('dG+geglu_bwd  2-kernel', lambda: K.geglu_bwd(K.matmul_nn(x512, w2), dh), 2 * M * 1408 * 512),
        ('dW  TN        2816x512x110592', lambda: K.matmul_tn(dh, x512), 2 * M * 512 * 2816),
        ('dW  TN s4     2816x512x110592', lambda: K.matmul_tn(dh, x512, split_k=4), 2 * M * 512 * 2816),
        ('dW  TN s40    512x512x110592', lambda: K.matmul_tn(x512, x512, split_k=40), 2 * M * 512 * 512),
        ('dW  TN        512x512x110592', lambda: K.matmul_tn(x512, x512), 2 * M * 512 * 512),
        ('sq  NT        8192x8192x8192', lambda: K.linear(sqa, sqb, out=sqo), 2 * 8192 ** 3),
        ('sq  NN        8192x8192x8192', lambda: K.matmul_nn(sqa, sqb), 2 * 8192 ** 3),
        ('sq  TN        8192x8192x8192', lambda: K.matmul_tn(sqa, sqb), 2 * 8192 ** 3),
    ]
    from ctclip_mi355x import _lib
    variants = [v for v in os.environ.get('GEMM_VARIANTS', '8,1').split(',')]
    only = [o for o in os.environ.get('GEMM_ONLY', '').split(',') if o]
    for name, fn, fl in cases:
        if only and not any(o in name for o in only):
            continue
        row = []
        for v in variants:   # '8' or '8s<stagger>', 'n' suffix = not persistent
            vv, _, st = v.rstrip('n').partition('s')
            _lib.lib().ctclip_gemm_set_persist(0 if v.endswith('n') else 1)
            _lib.lib().ctclip_gemm_set_variant(int(vv))
            _lib.lib().ctclip_gemm_set_stagger(int(st) if st else -1)
            ms = timeit(fn)
            row.append(f'v{v} {ms:7.3f} ms {fl / ms / 1e9:7.1f} TF/s')
        print(f'{name:34s} ' + ' | '.join(row), flush=True)
    _lib.lib().ctclip_gemm_set_variant(8)
    _lib.lib().ctclip_gemm_set_stagger(-1)
    _lib.lib().ctclip_gemm_set_persist(1)
    if os.environ.get('NO_LIB'):
        return
    # hipBLASLt (torch.matmul) on the same shapes, for a library reference point
    lib = [
        ('lib FF1 NT  110592x2816x512', lambda: torch.matmul(x512, w1.t()), 2 * M * 2816 * 512),
        ('lib FF2 NT  110592x512x1408', lambda: torch.matmul(x1408, w2.t()), 2 * M * 512 * 1408),
        ('lib Q   NT  110592x256x512', lambda: torch.matmul(x512, wq.t()), 2 * M * 256 * 512),
        ('lib dX  NN  110592x512x2816', lambda: torch.matmul(dh, w1), 2 * M * 512 * 2816),
        ('lib dW  TN  2816x512x110592', lambda: torch.matmul(dh.t(), x512), 2 * M * 512 * 2816),
        ('lib sq  NT  8192x8192x8192', lambda: torch.matmul(sq, sq.t()), 2 * 8192 ** 3),
    ]
    sq = r(8192, 8192)
    for name, fn, fl in lib:
        ms = timeit(fn)
        print(f'{name:34s} {ms:8.3f} ms  {fl / ms / 1e9:8.1f} TF/s', flush=True)


if __name__ == '__main__' and len(sys.argv) == 1:
    main()


def ksweep():
    """Per-tile fixed cost vs per-K-step cost: NT GEMM, M=27648, N=2816, K in 512..4096."""
    torch.manual_seed(0)
    Mm, N = 27648, 2816
    for Kd in (512, 1024, 2048, 4096):
        x = (torch.rand(Mm, Kd, device='cuda') * 2 - 1).bfloat16()
        w = (torch.rand(N, Kd, device='cuda') * 2 - 1).bfloat16()
        out = torch.empty(Mm, N, device='cuda', dtype=torch.bfloat16)
        ms = timeit(lambda: K.linear(x, w, out=out))
        print(f'NT M={Mm} N={N} K={Kd:5d}: {ms:7.3f} ms {2 * Mm * N * Kd / ms / 1e9:8.1f} TF/s', flush=True)


if __name__ == '__main__' and len(sys.argv) > 1 and sys.argv[1] == 'ksweep':
    ksweep()
