"""GPU diagnostic (round 5): the fp16 LayerNorm-fused to_out GEMM against the unfused pair at the
base B = 8 shape, the bf16 forms, PEG x32 at B = 8 against the bf16-tap kernel, and the layer-level
fused / unfused comparison with the fp16 forward on and off."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                                'ctpa-clip_amd'))
from ctclip_mi355x import kernels as K  # noqa: E402
from ctclip_mi355x import functional as Fn, attention as A  # noqa: E402


def rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30)).item()


g = torch.Generator(device='cuda').manual_seed(1)
for M in (16384, 110592):
    for dt in (torch.float16, torch.bfloat16):
        o = torch.randn(M, 256, device='cuda', generator=g).to(dt)
        W = (torch.randn(512, 256, device='cuda', generator=g) / 16).to(dt)
        res = torch.randn(M, 512, device='cuda', generator=g)
        gm = 1 + 0.1 * torch.randn(512, device='cuda', generator=g)
        bt = 0.1 * torch.randn(512, device='cuda', generator=g)
        with K.ln_guard():
            fu = K.linear_residual_ln(o, W, res, gm, bt, 1e-5, y16=(dt == torch.float16))
        sh = torch.empty(M, 512, device='cuda', dtype=torch.bfloat16)
        x2 = K.linear(o, W, residual=res, out_dtype=torch.float32, out2=sh)
        ln = K.layernorm_fwd(x2, gm, bt, 1e-5, out_f16=(dt == torch.float16))
        torch.cuda.synchronize()
        msg = f'M={M} {dt}: x1f {rel(fu[0], x2):.2e} x1b {rel(fu[1], sh):.2e} y {rel(fu[2], ln[0]):.2e} ' \
              f'mean {rel(fu[3], ln[2]):.2e} rstd {rel(fu[4], ln[3]):.2e}'
        if dt == torch.float16:
            msg += f' y16 {rel(fu[5], ln[4]):.2e}'
        print(msg, 'status', K.ln_fused_status(), flush=True)
B = 8
xf = torch.randn(B * 24 ** 3, 512, device='cuda', generator=g)
w = torch.randn(512, 27, device='cuda', generator=g) * 0.1
b = torch.randn(512, device='cuda', generator=g) * 0.1
for mode in (0, 1):
    of, ob, m, r = K.peg_fwd_stats(xf.bfloat16(), xf, B, 24, 24, 24, w, b, mode)
    of2, ob2, oh2, m2, r2 = K.peg_fwd_x32(xf, B, 24, 24, 24, w, b, mode, stats=True, want_f16=True)
    xr = xf.bfloat16().float()
    of3, _, _, _, _ = K.peg_fwd_x32(xr, B, 24, 24, 24, w, b, mode)
    print(f'PEG B=8 mode {mode}: x32 vs bf16-tap kernel on bf16-exact x {rel(of3, K.peg_fwd(xr.bfloat16(), xr, B, 24, 24, 24, w, b, mode)[0]):.2e}; '
          f'f32 x: out {rel(of2, of):.2e} mean {rel(m2, m):.2e} rstd {rel(r2, r):.2e}', flush=True)
torch.manual_seed(0)
tr = A.Transformer(512, depth=1, dim_head=32, heads=8).cuda()
with torch.no_grad():
    for p in tr.parameters():
        p.add_(0.02 * torch.randn_like(p))
for mode in (1, 0):
    geo = Fn.Geo(B=8, T=24, Hg=24, Wg=24, heads=8, dim_head=32, mode=mode)
    x0 = torch.randn(geo.M, 512, device='cuda')
    for f16 in (True, False):
        Fn.set_vit_f16(f16)
        ys = []
        for fused in (False, True):
            K.LN_FUSED = fused
            with torch.no_grad(), K.ln_guard():
                y, _ = tr.run(x0, x0.bfloat16(), geo)
            ys.append(y)
        torch.cuda.synchronize()
        print(f'layer mode {mode} f16={f16}: fused vs unfused {rel(ys[1], ys[0]):.2e}', flush=True)
K.LN_FUSED = True
Fn.set_vit_f16(True)
