"""Two GEMMs of one ViT layer's backward that do not depend on each other, serial on one stream vs
concurrent on two streams with the chip split by the persistent grid cap
(ctclip_gemm_set_grid_cap).  Pairs: GEGLU-backward dG (HBM-heavy epilogue) with the FF2 weight
gradient (MFMA-bound); the attention-out dX with its weight gradient.   usage: python tools/overlap_probe.py (GPU)"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'ctpa-clip_amd'))
import torch  # noqa: E402

from ctclip_mi355x import _lib, kernels as K  # noqa: E402

M = 110592


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


def main():
    torch.manual_seed(0)
    L = _lib.lib()
    r = lambda *s: (torch.rand(*s, device='cuda') * 2 - 1).bfloat16()  # noqa: E731
    dx3, g, h, w2 = r(M, 512), r(M, 1408), r(M, 2816), r(512, 1408)
    o, wo = r(M, 256), r(512, 256)
    side = torch.cuda.Stream()
    main_s = torch.cuda.current_stream()
    pairs = {
        'geglu_bwd | dW2': (lambda: K.matmul_nn_geglu_bwd(dx3, w2, h), lambda: K.matmul_tn(dx3, g)),
        'dX out    | dWo': (lambda: K.matmul_nn(dx3, wo), lambda: K.matmul_tn(dx3, o)),
    }
    for name, (fa, fb) in pairs.items():
        ta, tb = timeit(fa), timeit(fb)

        def serial():
            fa()
            fb()
        ts = timeit(serial)
        row = [f'{name}: A {ta:.3f}  B {tb:.3f}  serial {ts:.3f} ms']
        for ca, cb in ((128, 128), (160, 96), (192, 64), (96, 160)):
            def conc():
                ev = torch.cuda.Event()
                ev.record(main_s)
                side.wait_event(ev)
                L.ctclip_gemm_set_grid_cap(ca)
                fa()
                L.ctclip_gemm_set_grid_cap(cb)
                with torch.cuda.stream(side):
                    fb()
                L.ctclip_gemm_set_grid_cap(0)
                ev2 = torch.cuda.Event()
                ev2.record(side)
                main_s.wait_event(ev2)
            row.append(f'{ca}/{cb} {timeit(conc):.3f}')
        print(' | '.join(row), flush=True)


if __name__ == '__main__':
    main()
