"""Time the patchify + LayerNorm(4000) strip kernel at the bench size (B = 8 int16 volumes
240 x 480 x 480) with and without its XCD-aware block order (CTCLIP_PATCH_XCD, read at library
load, so each setting runs in its own child process; the parent never touches the GPU).
Reports ms per call and the HBM rate over the algorithmic bytes (int16 in + bf16 rows out).
usage: python tools/patch_ab.py   (GPU)"""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child():
    sys.path.insert(0, os.path.join(REPO, 'ctpa-clip_amd'))
    import torch
    from ctclip_mi355x import kernels as K
    from ctclip_mi355x.layers import patch_offsets
    B = 8
    vol = torch.randint(-1200, 1200, (B, 1, 240, 480, 480), device='cuda', dtype=torch.int16)
    offs = patch_offsets(1, 10, 20, 20, 480, 480).to('cuda')
    out = None
    for _ in range(3):
        out = K.patch_ln(vol, True, 10, 20, offs, ld=4032)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    times = []
    for _ in range(5):
        s.record()
        for _ in range(10):
            out = K.patch_ln(vol, True, 10, 20, offs, ld=4032)
        e.record()
        torch.cuda.synchronize()
        times.append(s.elapsed_time(e) / 10)
    ms = sorted(times)[2]
    nbytes = vol.numel() * 2 + out.numel() * 2
    print(f"CTCLIP_PATCH_XCD={os.environ.get('CTCLIP_PATCH_XCD', '1')}: {ms:.4f} ms  "
          f"{nbytes / ms / 1e6:.0f} GB/s over {nbytes / 1e9:.3f} GB", flush=True)


if __name__ == '__main__':
    if len(sys.argv) > 1 and sys.argv[1] == 'child':
        child()
    else:
        for v in ('0', '1', '0', '1'):
            env = dict(os.environ, CTCLIP_PATCH_XCD=v)
            r = subprocess.run([sys.executable, __file__, 'child'], env=env)
            if r.returncode != 0:
                sys.exit(r.returncode)
