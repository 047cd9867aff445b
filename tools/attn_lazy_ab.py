"""Spatial attention forward (base shape: 192 frames x 576 tokens x 8 heads, CPB bias) and BERT
attention (8 x 128 tokens, 12 heads of 64, key mask) with and without the lazy online-softmax
rescale (CTCLIP_ATTN_LAZY, read at library load: one child process per setting, the parent never
touches the GPU).  Prints median us per launch and the max |o| difference against the eager
rescale (setting 0) on the same seeded inputs.
usage: python tools/attn_lazy_ab.py   (GPU)"""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(out_path):
    sys.path.insert(0, os.path.join(REPO, 'ctpa-clip_amd'))
    import torch
    import torch.nn.functional as F
    from ctclip_mi355x import kernels as K
    torch.manual_seed(0)
    dev = 'cuda'
    res = {}
    # spatial, base shape
    B, T, gh, gw, H, D = 8, 24, 24, 24, 8, 32
    L, nseq = gh * gw, B * T
    M = nseq * L
    q = (F.normalize(torch.randn(M, H, D, device=dev), dim=-1) * 2.5).reshape(M, H * D).bfloat16()
    kv = torch.randn(M, 2 * H * D, device=dev)
    kv[:, :H * D] = (F.normalize(kv[:, :H * D].reshape(M, H, D), dim=-1) * 2.5).reshape(M, H * D)
    kv = kv.bfloat16()
    nb = (2 * gh - 1) * (2 * gw - 1)
    u = torch.randn(H, nb, device=dev) * 0.5
    args = dict(L=L, H=H, D=D, nseq=nseq, scale=8.0, seq=(1, L, 0, 1), bias_u=u, grid=(gh, gw))
    # BERT
    Bt, Lt, Ht, Dt = 8, 128, 12, 64
    Mt = Bt * Lt
    qt = (torch.randn(Mt, Ht * Dt, device=dev) * 0.5).bfloat16()
    kt = (torch.randn(Mt, Ht * Dt, device=dev) * 0.5).bfloat16()
    vt = torch.randn(Mt, Ht * Dt, device=dev).bfloat16()
    km = torch.ones(Bt, Lt, device=dev, dtype=torch.int32)
    km[:, 100:] = 0
    targs = dict(L=Lt, H=Ht, D=Dt, nseq=Bt, scale=0.125, seq=(1, Lt, 0, 1), kmask=km)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for name, fn in (('spatial', lambda: K.attn_fwd(q, kv[:, :H * D], kv[:, H * D:], **args)),
                     ('bert', lambda: K.attn_fwd(qt, kt, vt, **targs))):
        o, lse = fn()
        ts = []
        for _ in range(7):
            s.record()
            for _ in range(10):
                fn()
            e.record()
            torch.cuda.synchronize()
            ts.append(s.elapsed_time(e) * 100)   # us per launch
        res[name] = (sorted(ts)[3], o.float().cpu(), lse.cpu())
    torch.save(res, out_path)
    print(f"CTCLIP_ATTN_LAZY={os.environ.get('CTCLIP_ATTN_LAZY', '8')}: " +
          ', '.join(f'{k} {v[0]:.1f} us' for k, v in res.items()), flush=True)


if __name__ == '__main__':
    if len(sys.argv) > 2 and sys.argv[1] == 'child':
        child(sys.argv[2])
    else:
        import torch
        outs = {}
        # the padded-row (unswizzled) forward as an A/B library, when built:
        #   make -C ctpa-clip_amd/csrc OUT=../../tools/ab/libctclip_noswz.so OBJDIR=build_noswz EXTRA=-DCTCLIP_ATTN_FWD_SWZ=0
        noswz = os.path.join(REPO, 'tools', 'ab', 'libctclip_noswz.so')
        runs = [('0', {}), ('8', {}), ('8-noswz', {'CTCLIP_HIP_LIB': noswz}), ('0', {}), ('8', {}),
                ('8-noswz', {'CTCLIP_HIP_LIB': noswz}), ('4', {}), ('16', {})]
        for v, extra in runs:
            if 'CTCLIP_HIP_LIB' in extra and not os.path.exists(noswz):
                continue
            path = f'/tmp/attn_lazy_{v}.pt'
            env = dict(os.environ, CTCLIP_ATTN_LAZY=v.split('-')[0], **extra)
            print(f'[{v}]', end=' ', flush=True)
            r = subprocess.run([sys.executable, __file__, 'child', path], env=env)
            if r.returncode != 0:
                sys.exit(r.returncode)
            outs[v] = torch.load(path, weights_only=True)
        for v in [x for x in ('8', '8-noswz', '4', '16') if x in outs]:
            for k in ('spatial', 'bert'):
                do = (outs[v][k][1] - outs['0'][k][1]).abs().max().item()
                dl = (outs[v][k][2] - outs['0'][k][2]).abs().max().item()
                print(f'lazy {v} vs 0, {k}: max |do| {do:.3e}, max |dlse| {dl:.3e}')
