"""What does the erf cost inside the GEGLU epilogues?  Times FF1 + GEGLU and the fused GEGLU
backward at the bench shape with the product library and with a diagnostic build whose GELU is a
plain multiply (tools/ab/libctclip_cheapgelu.so: make -C ctpa-clip_amd/csrc
OUT=../../tools/ab/libctclip_cheapgelu.so OBJDIR=build_cheapgelu EXTRA=-DCTCLIP_DIAG_CHEAP_GELU --
WRONG activations, timing only), one child process per library, interleaved.
usage: python tools/gelu_cost_ab.py   (GPU)"""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child():
    sys.path.insert(0, os.path.join(REPO, 'ctpa-clip_amd'))
    import torch
    from ctclip_mi355x import kernels as K
    M = 110592
    torch.manual_seed(0)
    r = lambda *s: (torch.rand(*s, device='cuda') * 2 - 1).bfloat16()  # noqa: E731
    x512, h = r(M, 512), r(M, 2816)
    w1, w2 = r(2816, 512), r(512, 1408)
    g = torch.empty(M, 1408, device='cuda', dtype=torch.bfloat16)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    out = []
    for name, fn in (('FF1+GEGLU', lambda: K.linear(x512, w1, act=K.ACT_GEGLU, out2=g)),
                     ('GEGLU-bwd', lambda: K.matmul_nn_geglu_bwd(x512, w2, h))):
        fn()
        ts = []
        for _ in range(5):
            s.record()
            for _ in range(10):
                fn()
            e.record()
            torch.cuda.synchronize()
            ts.append(s.elapsed_time(e) / 10)
        out.append(f'{name} {sorted(ts)[2]:.4f} ms')
    lib = os.path.basename(os.environ.get('CTCLIP_HIP_LIB', 'libctclip_hip.so'))
    print(f'{lib:28s} ' + ', '.join(out), flush=True)


if __name__ == '__main__':
    if len(sys.argv) > 1 and sys.argv[1] == 'child':
        child()
    else:
        cheap = os.path.join(REPO, 'tools', 'ab', 'libctclip_cheapgelu.so')
        for _ in range(3):
            for extra in ({}, {'CTCLIP_HIP_LIB': cheap}):
                r = subprocess.run([sys.executable, __file__, 'child'], env=dict(os.environ, **extra))
                if r.returncode != 0:
                    sys.exit(r.returncode)
