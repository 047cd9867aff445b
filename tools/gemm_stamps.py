"""Per-tile timeline of the persistent 8-phase GEMM from s_memtime stamps (diagnostic build:
CTCLIP_HIP_LIB=.../libctclip_hip_stamps.so, compiled with -DCTCLIP_GEMM_STAMPS).
Stamps per (workgroup, tile): 0 tile start, 2 after the second K-tile, 3 after the last MFMA
(+ barrier), 4 after the epilogue's stores are issued, 5 tile start in s_memrealtime.
usage: python tools/gemm_stamps.py [shape ...]   (GPU)"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'ctpa-clip_amd'))
import torch  # noqa: E402

from ctclip_mi355x import _lib, kernels as K  # noqa: E402

M = 110592


def main():
    torch.manual_seed(0)
    r = lambda *s: (torch.rand(*s, device='cuda') * 2 - 1).bfloat16()  # noqa: E731
    x512, x1408 = r(M, 512), r(M, 1408)
    w1, w2 = r(2816, 512), r(512, 1408)
    g = torch.empty(M, 1408, device='cuda', dtype=torch.bfloat16)
    dh = torch.empty(M, 2816, device='cuda', dtype=torch.bfloat16)
    cb = r(8192, 512)
    cand = torch.empty(M, 128, 2, device='cuda')
    cand2 = torch.empty(M, 128, device='cuda')
    shapes = {
        'ff1': lambda: K.linear(x512, w1, act=K.ACT_GEGLU, out2=g),
        'ff1plain': lambda: K.linear(x512, w1, out=dh),
        'dx1408': lambda: K.matmul_nn(x512, w2),
        'geglubwd': lambda: K.matmul_nn_geglu_bwd(x512, w2, dh),
        'dwq': lambda: K.matmul_tn(x512[:, :256], x512),
        'vq': lambda: K.gemm_raw(M, 8192, 512, x512, 512, True, cb, 512, True, cand, 128, C2=cand2, ldc2=128,
                                 act=K.ACT_ARGMAX),
    }
    L = _lib.lib()
    L.ctclip_gemm_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    buf = np.zeros((256, 32, 6), dtype=np.uint64)
    for name in (sys.argv[1:] or ['ff1', 'ff1plain']):
        fn = shapes[name]
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        L.ctclip_gemm_stamps(buf.ctypes.data, 1)
        fn()
        torch.cuda.synchronize()
        assert L.ctclip_gemm_stamps(buf.ctypes.data, 1) == 0
        st = buf.astype(np.int64)
        valid = st[:, :, 4] > 0
        rows = []
        for wg in range(256):
            n = int(valid[wg].sum())
            for t in range(n):
                s = st[wg, t]
                nxt = st[wg, t + 1, 0] if t + 1 < n else s[4]
                rows.append((s[2] - s[0], s[3] - s[2], s[4] - s[3], nxt - s[4], 0, 0, t))
        a = np.array(rows, dtype=np.float64)
        first = a[a[:, 6] == 0]
        later = a[a[:, 6] > 0]
        if len(later) == 0:   # one tile per workgroup (split-K dW): report the first tiles
            later = first
        print(f'== {name}: {len(a)} tiles; median cycles per tile part (later tiles / first):')
        for k, lab in enumerate(['K-tiles 0-1', 'K-tiles 2..', 'epilogue issue', 'wait before next tile']):
            print(f'   {lab:34s} {np.median(later[:, k]):9.0f}  p90 {np.percentile(later[:, k], 90):9.0f}'
                  f'   first {np.median(first[:, k]):9.0f}')
        tot = later[:, :4].sum(1)
        print(f'   {"tile total":34s} {np.median(tot):9.0f}')
        # realtime (100 MHz, chip-wide) tile starts: how many workgroups are in their epilogue at once
        rt = st[:, :, 5]
        rt0 = rt[valid].min()
        for t in (0, 1, 4, 8, 12):
            v = rt[:, t][valid[:, t]] - rt0
            if len(v):
                print(f'   tile {t:2d} start (us, realtime) p0/25/50/75/100: ' +
                      ' '.join(f'{x / 100:.2f}' for x in np.percentile(v, [0, 25, 50, 75, 100])))


if __name__ == '__main__':
    main()
