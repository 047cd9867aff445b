"""MX-fp8 GEMM vs the build's bf16 GEMM at the 3D-ViT's linear shapes (B = 8: 110,592 tokens):
HIP-event time per launch and TFLOP/s (2MNK algorithmic flops; K = the layer's true K)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'ctpa-clip_amd'))
import torch  # noqa: E402

from ctclip_mi355x import kernels as K  # noqa: E402


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
    M = 110592
    for name, N, Kx in [('FF1 512->2730', 2730, 512), ('FF2 1365->512', 512, 1365), ('QKV 512->768', 768, 512),
                        ('out 256->512', 512, 256), ('square 4096', 4096, 4096)]:
        m = M if name != 'square 4096' else 4096
        kp = (Kx + 63) // 64 * 64                     # the build's padded leading dims
        x = torch.zeros(m, kp, device='cuda', dtype=torch.bfloat16)[:, :Kx]
        x.copy_(torch.randn(m, Kx, device='cuda'))
        w = torch.zeros(N, kp, device='cuda', dtype=torch.bfloat16)[:, :Kx]
        w.copy_(torch.randn(N, Kx, device='cuda') * Kx ** -0.5)
        qx, sx = K.quant_mxfp8(x)
        qw, sw = K.quant_mxfp8(w)
        c8 = torch.empty(m, (N + 7) // 8 * 8, device='cuda', dtype=torch.bfloat16)[:, :N]   # aligned ld
        t8s = []
        for tile in (128, 256):
            K.gemm_mxfp8_set_tile(tile)
            t8s.append(timeit(lambda: K.gemm_mxfp8(qx, sx, qw, sw, out=c8)))
        K.gemm_mxfp8_set_tile(0)
        t8 = timeit(lambda: K.gemm_mxfp8(qx, sx, qw, sw, out=c8))
        tq = timeit(lambda: K.quant_mxfp8(x))
        # the bf16 kernel needs K, N % 8: it runs on the zero-padded operands (as the model's layers do)
        n8 = (N + 7) // 8 * 8
        xb = x.as_strided((m, kp), (kp, 1))
        wb = torch.zeros(n8, kp, device='cuda', dtype=torch.bfloat16)
        wb[:N] = w.as_strided((N, kp), (kp, 1))
        cb = torch.empty(m, n8, device='cuda', dtype=torch.bfloat16)
        tb = timeit(lambda: K.linear(xb, wb, out=cb))
        fl = 2.0 * m * N * Kx
        print(f'{name:16s} M={m:6d}  mxfp8 {t8 * 1e3:8.1f} us {fl / t8 / 1e9:7.1f} TF/s '
              f'(tile 128: {fl / t8s[0] / 1e9:6.1f}, 256: {fl / t8s[1] / 1e9:6.1f}) | quant(x) {tq * 1e3:7.1f} us '
              f'| bf16 build {tb * 1e3:8.1f} us {fl / tb / 1e9:7.1f} TF/s', flush=True)


if __name__ == '__main__':
    main()
