"""Weight-gradient (split-K, reduction over the 110,592 tokens) GEMM shapes of the 3D-ViT step on the
three large-tile kernel variants (ctclip_gemm_set_variant: 8 = 8-phase 256x256x64, one workgroup
per CU; 1 = 128x256x32, two workgroups per CU; 2 = 256x256x32 4-slot ring), at the split the
library picks and at 2x / 0.5x that split.  The dW GEMMs are the step's largest kernel family
(41 launches, ~5.5 ms) and run at ~45 % MFMA busy with HBM at ~2.6 TB/s: latency-bound.
Interleaved rounds in one process; median ms of the GEMM + slab reduction.
usage: python tools/dw_variant_ab.py   (GPU)"""
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'ctpa-clip_amd'))
import torch  # noqa: E402

from ctclip_mi355x import kernels as K, _lib  # noqa: E402

M = 110592


def timeit(fn, n=8):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


def auto_split(N, Kd):
    t256 = ((N + 255) // 256) * ((Kd + 255) // 256)
    return max(1, 256 // t256)


def main():
    torch.manual_seed(0)
    r = lambda *s: (torch.rand(*s, device='cuda') * 2 - 1).bfloat16()  # noqa: E731
    acts = {n: r(M, n) for n in (256, 512, 768, 1408, 2816)}
    shapes = {'FF1 2816x512': (2816, 512), 'FF2 512x1408': (512, 1408), 'KV 512x512': (512, 512),
              'Q 256x512': (256, 512), 'Wo 512x256': (512, 256)}
    L = _lib.lib()
    confs = []
    for v in (8, 1, 2):
        for f in (1.0, 2.0, 0.5):
            confs.append((v, f))
    res = {(sh, c): [] for sh in shapes for c in confs}
    outs = {}
    for rnd in range(3):
        for (v, f) in confs:
            L.ctclip_gemm_set_variant(v)
            for sh, (N, Kd) in shapes.items():
                s = max(1, int(round(auto_split(N, Kd) * f)))
                dy, x = acts[N], acts[Kd]
                out = torch.empty(N, Kd, device='cuda')
                res[(sh, (v, f))].append(timeit(lambda: K.matmul_tn(dy, x, out=out, split_k=s)))
                if rnd == 0:
                    outs[(sh, v, f)] = out.clone()
        print(f'round {rnd} done', flush=True)
    L.ctclip_gemm_set_variant(8)
    for sh in shapes:
        base = outs[(sh, 8, 1.0)]
        for (v, f) in confs:
            d = (outs[(sh, v, f)] - base).abs().max().item() / base.abs().max().item()
            assert d < 1e-4, (sh, v, f, d)
    print('median ms (GEMM + slab reduction); columns (variant, split factor x auto)')
    print('%-14s' % 'shape' + ''.join('%10s' % ('%d,%.1f' % c) for c in confs))
    for sh, (N, Kd) in shapes.items():
        fl = 2.0 * M * N * Kd
        row = '%-14s' % sh + ''.join('%10.4f' % statistics.median(res[(sh, c)]) for c in confs)
        best = min(confs, key=lambda c: statistics.median(res[(sh, c)]))
        print(row + '   best %s %.0f TF/s' % (best, fl / statistics.median(res[(sh, best)]) / 1e9), flush=True)


if __name__ == '__main__':
    main()
