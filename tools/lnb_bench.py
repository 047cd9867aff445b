"""Isolated LayerNorm-backward timing at the step's shape (110,592 x 512: bf16 dy / x, f32 dres,
f32 + bf16 dx, gamma / beta partials); the library comes from CTCLIP_HIP_LIB when set (A/B)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'ctpa-clip_amd'))
import torch  # noqa: E402

from ctclip_mi355x import kernels as K  # noqa: E402


def main():
    M, D = 110592, 512
    torch.manual_seed(0)
    dy = torch.randn(M, D, device='cuda').bfloat16()
    x = torch.randn(M, D, device='cuda').bfloat16()
    dres = torch.randn(M, D, device='cuda')
    g = torch.randn(D, device='cuda')
    _, _, mean, rstd = K.layernorm_fwd(x.float(), g, g, 1e-5)
    dg, db = torch.zeros(D, device='cuda'), torch.zeros(D, device='cuda')

    def run():
        K.layernorm_bwd(dy, x, mean, rstd, g, dres=dres, dgamma_out=dg, dbeta_out=db)
    for _ in range(5):
        run()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(50):
        run()
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / 50 * 1e3
    gb = M * D * (2 + 2 + 4 + 4 + 2) / 1e9
    print(f'{os.path.basename(os.environ.get("CTCLIP_HIP_LIB", "libctclip_hip.so"))}: layernorm_bwd {us:.1f} us '
          f'(incl. partial reduction), {gb / us * 1e6 / 1e3:.2f} TB/s on {gb:.3f} GB')


if __name__ == '__main__':
    main()
