"""Per-call census of the contrastive step's GEMMs (shape, operand layouts, epilogue, stream) with
HIP-event durations, on the stream each GEMM is launched on.
usage: python tools/gemm_census.py   (GPU)"""
import collections
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'ctpa-clip_amd'))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    from ctclip_mi355x import kernels as K
    from ctclip_mi355x.models import build_ctclip, set_finetune_trainable
    from ctclip_mi355x.trainer import CTClipTrainer
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    model = set_finetune_trainable(build_ctclip()).to(dev)
    tr = CTClipTrainer(model)
    hu, text = bench.synthetic_inputs(8, 128, 0, dev)
    for _ in range(3):
        tr.train_step(text, hu)
    torch.cuda.synchronize()
    rec = []
    orig = K._gemm_raw

    def timed(M, N, Kd, A, lda, akc, B, ldb, bkc, C, ldc, **kw):
        st = torch.cuda.current_stream()
        e0 = st.record_event(torch.cuda.Event(enable_timing=True))
        orig(M, N, Kd, A, lda, akc, B, ldb, bkc, C, ldc, **kw)
        e1 = st.record_event(torch.cuda.Event(enable_timing=True))
        key = (M, N, Kd, int(akc), int(bkc), kw.get('act', 0), kw.get('R') is not None,
               C.dtype == torch.float32, kw.get('C2') is not None, kw.get('split_k', 1), st.stream_id != 0)
        rec.append((key, e0, e1))

    K._gemm_raw = timed
    tr.train_step(text, hu)
    torch.cuda.synchronize()
    K._gemm_raw = orig
    agg = collections.OrderedDict()
    for key, e0, e1 in rec:
        t = e0.elapsed_time(e1)
        a = agg.setdefault(key, [0, 0.0])
        a[0] += 1
        a[1] += t
    tot = {False: 0.0, True: 0.0}
    print(f'{"M":>7} {"N":>6} {"K":>7} kc(A,B) act R f32 C2 split side  calls  ms/call  ms  TF/s')
    for key, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        M, N, Kd, akc, bkc, act, r, f32, c2, sk, side = key
        tot[side] += t
        print(f'{M:7d} {N:6d} {Kd:7d}   {akc}{bkc}    {act:3d} {int(r)} {int(f32):3d} {int(c2):2d} {sk:5d} {int(side):4d} '
              f'{n:6d} {t / n:8.3f} {t:6.3f} {2.0 * M * N * Kd * n / (t * 1e-3) / 1e12:6.1f}')
    print(f'total: main stream {tot[False]:.3f} ms, side streams {tot[True]:.3f} ms')


if __name__ == '__main__':
    main()
