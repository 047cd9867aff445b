"""GPU micro-benchmark: the PEG forward and input-gradient kernels at the base shape (B = 8, 24^3 tokens, d = 512) --
the bf16-tap kernel (ctclip_peg_fwd_stats) against the f32-tap kernel (ctclip_peg_fwd_x32) for
both transformers' maps -- and the image projection (skinny streaming GEMM vs the split-K tile).
HIP events around 20 launches each; prints us per launch.  CTCLIP_HIP_LIB selects a library."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'ctpa-clip_amd'))
from ctclip_mi355x import kernels as K  # noqa: E402


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000 / reps


B, T, D = 8, 24, 512
M = B * T ** 3
torch.manual_seed(0)
xf = torch.randn(M, D, device='cuda')
xb = xf.bfloat16()
w = torch.randn(D, 1, 3, 3, 3, device='cuda') * 0.2
b = torch.randn(D, device='cuda') * 0.1
for mode in (0, 1):
    t_old = timeit(lambda: K.peg_fwd_stats(xb, xf, B, T, T, T, w, b, mode))
    t_new = timeit(lambda: K.peg_fwd_x32(xf, B, T, T, T, w, b, mode, stats=True))
    print(f'PEG fwd mode {mode}: bf16 taps {t_old:.1f} us, f32 taps {t_new:.1f} us', flush=True)
    dxf, dxb = torch.empty_like(xf), torch.empty_like(xb)
    t_bo = timeit(lambda: K.call('ctclip_peg_bwd_data', K.ptr(xb), K.ptr(xf), B, T, T, T, D, K.ptr(w), mode,
                                 K.ptr(dxf), K.ptr(dxb), K.stream_ptr()))
    t_bn = timeit(lambda: K.call('ctclip_peg_bwd_data_x32', K.ptr(xf), B, T, T, T, D, K.ptr(w), mode,
                                 K.ptr(dxf), K.ptr(dxb), K.stream_ptr()))
    print(f'PEG bwd data mode {mode}: bf16 taps {t_bo:.1f} us, f32 taps {t_bn:.1f} us', flush=True)
Kd, N = 294912, 512
pb = torch.randn(B, Kd, device='cuda').bfloat16()
Wb = (torch.randn(N, Kd, device='cuda') * 0.002).bfloat16()
t_sk = timeit(lambda: K.skinny_linear(pb, Wb))
split = max(1, min(512, Kd // 1024))


def splitk():
    slabs = torch.empty(split, B, N, device='cuda')
    K.gemm_raw(B, N, Kd, pb, Kd, True, Wb, Kd, True, slabs, N, split_k=split)
    out = torch.empty(B, N, device='cuda')
    K.reduce_slabs(slabs, out)


t_tile = timeit(splitk)
print(f'image projection 8 x 294912 x 512: skinny {t_sk:.1f} us ({Wb.numel() * 2 / t_sk / 1e6:.2f} TB/s), '
      f'split-K tile {t_tile:.1f} us', flush=True)
