"""A/B of the 8-phase GEMM's bf16 / GEGLU epilogue stores: straight from the transposed accumulator
(16 rows x 64 B per wave store, ~16 B/cycle per CU) or re-laid through the wave's LDS scratch so
consecutive lanes write consecutive 16 B of a row (~57 B/cycle per CU, profiles/r04c_store_probe.log),
each with a few start staggers (a desynchronised chip can use the faster per-CU drain).  Interleaved
rounds in one process; median ms.
usage: python tools/epi_lds_ab.py   (GPU)"""
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'ctpa-clip_amd'))
import torch  # noqa: E402

from ctclip_mi355x import kernels as K, _lib  # noqa: E402

M = 110592


def timeit(fn, n=10):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


def main():
    torch.manual_seed(0)
    r = lambda *s: (torch.rand(*s, device='cuda') * 2 - 1).bfloat16()  # noqa: E731
    x512, dh = r(M, 512), r(M, 2816)
    w1, wq, wkv = r(2816, 512), r(256, 512), r(512, 512)
    g = torch.empty(M, 1408, device='cuda', dtype=torch.bfloat16)
    cases = {
        'FF1+GEGLU': lambda: K.linear(x512, w1, act=K.ACT_GEGLU, out2=g),
        'FF1 plain': lambda: K.linear(x512, w1, out=dh),
        'KV bf16': lambda: K.linear(x512, wkv),
        'Q bf16': lambda: K.linear(x512, wq),
        'dX K=2816': lambda: K.matmul_nn(dh, w1),
    }
    L = _lib.lib()
    confs = [(lds, st) for lds in (0, 3, 2) for st in (0, 8)]
    res_ms = {(c, cf): [] for c in cases for cf in confs}
    for rnd in range(4):
        for cf in confs:
            L.ctclip_gemm_set_epi_lds(cf[0])
            L.ctclip_gemm_set_stagger(cf[1])
            for c, fn in cases.items():
                res_ms[(c, cf)].append(timeit(fn))
        print(f'round {rnd} done', flush=True)
    L.ctclip_gemm_set_stagger(-1)
    L.ctclip_gemm_set_epi_lds(0)
    print('median ms over 4 interleaved rounds; columns (epi_lds, stagger)')
    print('%-12s' % 'case' + ''.join('%11s' % ('%d,%d' % cf) for cf in confs))
    for c in cases:
        print('%-12s' % c + ''.join('%11.4f' % statistics.median(res_ms[(c, cf)]) for cf in confs), flush=True)


if __name__ == '__main__':
    main()
