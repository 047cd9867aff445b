"""Temporal (short-sequence) attention kernels at the base config, for library A/Bs:
  python tools/attn_small_ab.py dump <out.pt>     -- forward (O, fp16 O, lse) and backward (dQ, dK, dV)
                                                    of the library CTCLIP_HIP_LIB names, seeded inputs
  python tools/attn_small_ab.py cmp <a.pt> <b.pt> -- bit-for-bit comparison of two dumps
  python tools/attn_small_ab.py time              -- forward / backward microseconds
  python tools/attn_small_ab.py dumpfwd <out.pt>  -- spatial (CPB bias) and BERT-shape forwards (O, fp16 O, lse)
  python tools/attn_small_ab.py timefwd           -- spatial forward microseconds (with the fp16 copy)
  python tools/attn_small_ab.py dumpbwd <out.pt>  -- spatial (CPB bias) backward: dQ, dK, dV, bias gradient
  python tools/attn_small_ab.py timebwd           -- spatial backward microseconds
Q | K | V live in one [M, 768] buffer (the layers' packed projection), as in the step."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'ctpa-clip_amd'))
import torch  # noqa: E402


def setup():
    from ctclip_mi355x import kernels as K
    torch.manual_seed(0)
    B, T, Hg, Wg, H, D = 8, 24, 24, 24, 8, 32
    hw = Hg * Wg
    M = B * T * hw
    do = (torch.randn(M, H * D, device='cuda') * 0.3).bfloat16()
    kw = dict(L=T, H=H, D=D, nseq=B * hw, scale=8.0, seq=(hw, T * hw, 1, hw))
    if os.environ.get('LAYOUT', 'packed') == 'packed':
        qkv = (torch.randn(M, 3 * H * D, device='cuda') * 0.3).bfloat16()
        q, k, v = qkv[:, :H * D], qkv[:, H * D:2 * H * D], qkv[:, 2 * H * D:]
    else:   # three [M, 256] tensors
        q, k, v = [(torch.randn(M, H * D, device='cuda') * 0.3).bfloat16() for _ in range(3)]
    return K, q, k, v, do, kw


def run(K, q, k, v, do, kw):
    o, lse, o16 = K.attn_fwd(q, k, v, want_o16=True, **kw)
    dq, dk, dv = torch.empty_like(do), torch.empty_like(do), torch.empty_like(do)
    K.attn_bwd(q, k, v, o, lse, do, dq, dk, dv, **kw)
    return dict(o=o, o16=o16, lse=lse, dq=dq, dk=dk, dv=dv)


def main():
    mode = sys.argv[1]
    if mode == 'cmp':
        a, b = torch.load(sys.argv[2], weights_only=True), torch.load(sys.argv[3], weights_only=True)
        bad = [n for n in a if not torch.equal(a[n], b[n])]
        print('bit-identical' if not bad else f'DIFFER: {bad}', flush=True)
        sys.exit(1 if bad else 0)
    if mode in ('dumpfwd', 'timefwd', 'dumpbwd', 'timebwd'):
        return fwd_modes(mode)
    K, q, k, v, do, kw = setup()
    if mode == 'dump':
        out = run(K, q, k, v, do, kw)
        torch.save({n: t.cpu() for n, t in out.items()}, sys.argv[2])
        print('dumped', sys.argv[2], flush=True)
        return
    from gemm_bench import timeit
    o16 = os.environ.get('O16', '1') != '0'
    o, lse = K.attn_fwd(q, k, v, **kw)
    dq, dk, dv = torch.empty_like(do), torch.empty_like(do), torch.empty_like(do)
    f = timeit(lambda: K.attn_fwd(q, k, v, want_o16=o16, **kw), n=50)
    b = timeit(lambda: K.attn_bwd(q, k, v, o, lse, do, dq, dk, dv, **kw), n=50)
    print(f'temporal fwd {f * 1e3:7.1f} us  bwd {b * 1e3:7.1f} us  (layout {os.environ.get("LAYOUT", "packed")}, '
          f'fp16 copy {int(o16)})', flush=True)


def fwd_modes(mode):
    from ctclip_mi355x import kernels as K
    torch.manual_seed(1)
    B, T, G, H, D = 8, 24, 24, 8, 32
    L = G * G
    M = B * T * L
    r = lambda *s: (torch.randn(*s, device='cuda') * 0.3).bfloat16()  # noqa: E731
    q, kv = r(M, H * D), r(M, 2 * H * D)
    bias = torch.randn(H, (2 * G - 1) ** 2, device='cuda') * 0.5
    sp = dict(L=L, H=H, D=D, nseq=B * T, scale=8.0, seq=(1, L, 0, 1), bias_u=bias, grid=(G, G))
    if mode in ('dumpbwd', 'timebwd'):
        o, lse = K.attn_fwd(q, kv[:, :H * D], kv[:, H * D:], **sp)
        do = r(M, H * D)
        dq, dkv = torch.empty_like(q), torch.empty_like(kv)
        du = torch.zeros_like(bias)

        def bwd():
            du.zero_()
            K.attn_bwd(q, kv[:, :H * D], kv[:, H * D:], o, lse, do, dq, dkv[:, :H * D], dkv[:, H * D:],
                       dbias_u=du, **sp)
        if mode == 'timebwd':
            from gemm_bench import timeit
            print(f'spatial bwd {timeit(bwd, n=20) * 1e3:7.1f} us', flush=True)
            return
        bwd()
        torch.save({n: t.cpu() for n, t in dict(dq=dq, dkv=dkv, du=du).items()}, sys.argv[2])
        print('dumped', sys.argv[2], flush=True)
        return
    if mode == 'timefwd':
        from gemm_bench import timeit
        f = timeit(lambda: K.attn_fwd(q, kv[:, :H * D], kv[:, H * D:], want_o16=True, **sp), n=30)
        print(f'spatial fwd {f * 1e3:7.1f} us (fp16 copy 1)', flush=True)
        return
    o, lse, o16 = K.attn_fwd(q, kv[:, :H * D], kv[:, H * D:], want_o16=True, **sp)
    Lb, Hb, Db, Bb = 128, 12, 64, 8
    qkv = r(Bb * Lb, 3 * Hb * Db)
    lens = torch.tensor([128, 77, 5, 128, 64, 100, 1, 128])
    km = (torch.arange(Lb)[None, :] < lens[:, None]).int().cuda()
    bo, blse = K.attn_fwd(qkv[:, :Hb * Db], qkv[:, Hb * Db:2 * Hb * Db], qkv[:, 2 * Hb * Db:], L=Lb, H=Hb, D=Db,
                          nseq=Bb, scale=1 / 8, seq=(1, Lb, 0, 1), kmask=km)
    torch.save({n: t.cpu() for n, t in dict(o=o, o16=o16, lse=lse, bo=bo, blse=blse).items()}, sys.argv[2])
    print('dumped', sys.argv[2], flush=True)


if __name__ == '__main__':
    main()
