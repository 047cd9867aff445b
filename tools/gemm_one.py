"""Run one GEMM shape of the step repeatedly (for rocprofv3 counter passes).
usage: python tools/gemm_one.py {ff1,ff1h16,ff1plain,ff2,dxnn,dwtn,dx1408,geglubwd,dwq} [reps]
(ff1h16: the step's default FF1, fp16 operands and h, GEGLU epilogue)"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'ctpa-clip_amd'))
import torch  # noqa: E402

from ctclip_mi355x import kernels as K  # noqa: E402

M = 110592


def main():
    which = sys.argv[1]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    torch.manual_seed(0)
    r = lambda *s: (torch.rand(*s, device='cuda') * 2 - 1).bfloat16()  # noqa: E731
    x512, x1408 = r(M, 512), r(M, 1408)
    w1, w2 = r(2816, 512), r(512, 1408)
    g = torch.empty(M, 1408, device='cuda', dtype=torch.bfloat16)
    res = torch.randn(M, 512, device='cuda')
    dh = r(M, 2816)
    x512h, w1h = x512.half(), w1.half()
    fn = {
        'ff1': lambda: K.linear(x512, w1, act=K.ACT_GEGLU, out2=g),
        'ff1h16': lambda: K.linear(x512h, w1h, act=K.ACT_GEGLU, out2=g, out_dtype=K.F16),
        'ff1plain': lambda: K.linear(x512, w1, out=dh),
        'ff2': lambda: K.linear(x1408, w2, residual=res, out_dtype=torch.float32),
        'dxnn': lambda: K.matmul_nn(dh, w1),
        'dwtn': lambda: K.matmul_tn(dh, x512),
        'dx1408': lambda: K.matmul_nn(x512, w2),
        'geglubwd': lambda: K.matmul_nn_geglu_bwd(x512, w2, dh),
        'dwq': lambda: K.matmul_tn(x512[:, :256], x512),
    }[which]
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()


if __name__ == '__main__':
    main()
