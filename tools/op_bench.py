"""Isolated timing of the bandwidth-bound kernels at the step's shapes (110,592 tokens x 512)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'ctpa-clip_amd'))
import torch  # noqa: E402

from ctclip_mi355x import kernels as K  # noqa: E402

M, D = 110592, 512


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
    xf = torch.randn(M, D, device='cuda')
    xb = xf.bfloat16()
    g = torch.randn(D, device='cuda')
    b = torch.randn(D, device='cuda')
    _, _, mean, rstd = K.layernorm_fwd(xf, g, b, 1e-5)
    w = torch.randn(D, 1, 3, 3, 3, device='cuda') * 0.1
    pb = torch.randn(D, device='cuda')
    dg = torch.randn(M, 1408, device='cuda').bfloat16()
    h = torch.randn(M, 2816, device='cuda').bfloat16()
    qs = torch.ones(32, device='cuda')
    dxf, dxb = torch.empty_like(xf), torch.empty_like(xb)
    from ctclip_mi355x.preprocess import ct_volume_to_tensor
    scan = torch.randint(-1100, 2000, (512, 512, 300), device='cuda', dtype=torch.int16)
    vol = torch.empty(1, 240, 480, 480, device='cuda')
    ap, ag, am, av = (torch.rand(23_400_000, device='cuda') for _ in range(4))
    apb, acoef = torch.empty(23_400_000, device='cuda', dtype=torch.bfloat16), torch.ones(2, device='cuda')
    sl1024, r512 = torch.randn(1024, 1, 512, device='cuda'), torch.empty(1, 512, device='cuda')
    sl256, r768 = torch.randn(256, 1, 768, device='cuda'), torch.empty(1, 768, device='cuda')
    cases = [
        ('resample 512x512x300 i16 -> 240x480x480 (f64)',
         lambda: ct_volume_to_tensor(scan, 1.0, -1024.0, 0.7, 1.25, out=vol), scan.numel() * 2 + vol.numel() * 4),
        ('ln_fwd f32->bf16', lambda: K.layernorm_fwd(xf, g, b, 1e-5), M * D * 6),
        ('ln_fwd f32->bf16+f32', lambda: K.layernorm_fwd(xf, g, b, 1e-5, out_f32=True), M * D * 10),
        ('ln_bwd', lambda: K.layernorm_bwd(xb, xb, mean, rstd, g, dres=xf), M * D * (2 + 2 + 4 + 4 + 2)),
        ('peg_fwd mode0', lambda: K.peg_fwd(xb, xf, 8, 24, 24, 24, w, pb, 0), M * D * (2 + 4 + 4 + 2)),
        ('peg_fwd mode1', lambda: K.peg_fwd(xb, xf, 8, 24, 24, 24, w, pb, 1), M * D * (2 + 4 + 4 + 2)),
        ('peg_bwd (data+w)', lambda: K.peg_bwd(xb, xf, xb, 8, 24, 24, 24, w, 0), M * D * (2 + 4 + 4 + 2 + 4)),
        ('peg_bwd mode1 (data+w)', lambda: K.peg_bwd(xb, xf, xb, 8, 24, 24, 24, w, 1), M * D * (2 + 4 + 4 + 2 + 4)),
        ('peg_bwd data only', lambda: K.call('ctclip_peg_bwd_data', K.ptr(xb), K.ptr(xf), 8, 24, 24, 24, D,
                                             K.ptr(w), 0, K.ptr(dxf), K.ptr(dxb), K.stream_ptr()),
         M * D * (2 + 4 + 4 + 2)),
        ('geglu_bwd', lambda: K.geglu_bwd(dg, h), M * (1408 + 2816 + 2816) * 2),
        ('l2n_fwd', lambda: K.l2norm_scale_fwd(xb[:, :256], 8, 32, qs), M * 256 * 4),
        ('l2n_bwd', lambda: K.l2norm_scale_bwd(xb[:, :256], xb[:, 256:], 8, 32, qs, dxb[:, :256]), M * 256 * 6),
        ('cast f32->bf16', lambda: K.cast_bf16(xf), M * D * 6),
        ('colsum bf16', lambda: K.colsum(xb), M * D * 2),
        ('adam 23.4M (+bf16 copy)', lambda: K.adam(ap, ag, am, av, lr=1e-4, b1=0.9, b2=0.99, eps=1e-8, wd=0.0, step=3,
                                                  coef=acoef, p_bf16=apb), 23_400_000 * 30),
        ('adam 23.4M', lambda: K.adam(ap, ag, am, av, lr=1e-4, b1=0.9, b2=0.99, eps=1e-8, wd=0.0, step=3,
                                      coef=acoef), 23_400_000 * 28),
        ('reduce 1024 slabs x 512', lambda: K.reduce_slabs(sl1024, r512), 1024 * 512 * 4),
        ('reduce 256 slabs x 768', lambda: K.reduce_slabs(sl256, r768), 256 * 768 * 4),
    ]
    from ctclip_mi355x import layers
    vol = torch.randint(-1200, 1201, (8, 1, 240, 480, 480), device='cuda', dtype=torch.int32).to(torch.int16)
    offs = layers.patch_offsets(1, 10, 20, 20, 480, 480).cuda()
    cases.append(('patch_ln int16->bf16', lambda: K.patch_ln(vol, True, 10, 20, offs), vol.numel() * 4))
    only = [o for o in os.environ.get('OP_ONLY', '').split(',') if o]
    for name, fn, nbytes in cases:
        if only and not any(o in name for o in only):
            continue
        ms = timeit(fn)
        print(f'{name:24s} {ms * 1e3:9.1f} us  {nbytes / ms / 1e9:7.2f} TB/s (algorithmic bytes)', flush=True)


if __name__ == '__main__':
    main()
