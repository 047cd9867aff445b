"""Bitwise A/B of every GEMM call of one B = 8 contrastive train step: the working-tree library
against libctclip_hip_old.so (tools/ab_build.sh) on identical inputs, each call serialised.
Prints the shape of every call before it runs (so a fault names its GEMM) and every mismatch.
usage: python tools/gemm_ab_check.py [batch]   (GPU)"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'ctpa-clip_amd'))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from ctclip_mi355x import kernels as K, _lib  # noqa: E402

OLD = ctypes.CDLL(os.path.join(REPO, 'ctpa-clip_amd', 'ctclip_mi355x', 'libctclip_hip_old.so'))
for _n, _a in _lib._SIGS.items():
    if hasattr(OLD, _n):
        getattr(OLD, _n).argtypes = _a
        getattr(OLD, _n).restype = ctypes.c_int32
orig = K._gemm_raw
stats = {'calls': 0, 'mismatch': 0}


def checked(M, N, K_, A, lda, a_kcontig, B, ldb, b_kcontig, C, ldc, **kw):
    stats['calls'] += 1
    tag = f'#{stats["calls"]} M={M} N={N} K={K_} a_kc={int(a_kcontig)} b_kc={int(b_kcontig)} ' + \
          ' '.join(f'{k}={v}' for k, v in kw.items() if k in ('act', 'split_k', 'batch', 'accumulate') and v)
    print(tag, flush=True)
    torch.cuda.synchronize()
    C2 = kw.get('C2')
    snap = [C.clone()] + ([C2.clone()] if C2 is not None else [])
    orig(M, N, K_, A, lda, a_kcontig, B, ldb, b_kcontig, C, ldc, **kw)
    torch.cuda.synchronize()
    new = [C.clone()] + ([C2.clone()] if C2 is not None else [])
    C.copy_(snap[0])
    if C2 is not None:
        C2.copy_(snap[1])
    # the same call through the old library (same argument struct)
    saved = _lib.lib
    _lib._LIB, keep = OLD, _lib._LIB
    try:
        _lib.lib = lambda: OLD
        orig(M, N, K_, A, lda, a_kcontig, B, ldb, b_kcontig, C, ldc, **kw)
    finally:
        _lib.lib = saved
        _lib._LIB = keep
    torch.cuda.synchronize()
    old = [C] + ([C2] if C2 is not None else [])
    for i, (a, b) in enumerate(zip(new, old)):
        if not torch.equal(a, b):
            stats['mismatch'] += 1
            d = (a.float() - b.float()).abs()
            print(f'   MISMATCH out{i}: max |d| {d.max().item():.3e}, {int((d > 0).sum())} of {d.numel()} differ, '
                  f'nan new {int(torch.isnan(a.float()).sum())} old {int(torch.isnan(b.float()).sum())}', flush=True)


def main():
    K._gemm_raw = checked
    from bench import synthetic_inputs
    from ctclip_mi355x.models import build_ctclip, set_finetune_trainable
    from ctclip_mi355x.trainer import CTClipTrainer
    b = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    dev = torch.device('cuda')
    torch.manual_seed(0)
    model = set_finetune_trainable(build_ctclip()).to(dev)
    model.train()
    tr = CTClipTrainer(model)
    hu, text = synthetic_inputs(b, 128, 0, dev)
    for step in range(2):
        loss = tr.train_step(text, hu)
        torch.cuda.synchronize()
        print(f'step {step}: loss {float(loss):.5f}; calls {stats["calls"]}, mismatches {stats["mismatch"]}',
              flush=True)


if __name__ == '__main__':
    main()
