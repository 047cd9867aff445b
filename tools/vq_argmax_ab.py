"""VQ distance GEMM + argmax epilogue (110,592 x 8,192 x 512, act 3) with the working-tree library
against libctclip_hip_old.so (tools/ab_build.sh): median ms over interleaved rounds (one child
process per library and round, the parent never touches the GPU) and bit-equality of the
(best, index) candidates and second-best scores between the libraries.
usage: python tools/vq_argmax_ab.py   (GPU)"""
import os
import statistics
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(REPO, 'ctpa-clip_amd', 'ctclip_mi355x')


def child(out):
    sys.path.insert(0, os.path.join(REPO, 'ctpa-clip_amd'))
    import torch
    from ctclip_mi355x import kernels as K
    torch.manual_seed(0)
    M = 110592
    x = torch.nn.functional.normalize(torch.randn(M, 512, device='cuda'), dim=-1).bfloat16()
    cb = torch.nn.functional.normalize(torch.randn(8192, 512, device='cuda'), dim=-1).bfloat16()
    cand = torch.empty(M, 128, 2, device='cuda')
    cand2 = torch.empty(M, 128, device='cuda')
    run = lambda: K.gemm_raw(M, 8192, 512, x, 512, True, cb, 512, True, cand, 128, C2=cand2, ldc2=128,  # noqa: E731
                             act=K.ACT_ARGMAX)
    for _ in range(3):
        run()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(20):
        run()
    e.record()
    torch.cuda.synchronize()
    torch.save({'ms': s.elapsed_time(e) / 20, 'cand': cand.cpu(), 'cand2': cand2.cpu()}, out)


def main():
    if len(sys.argv) > 1:
        child(sys.argv[1])
        return
    import torch
    res = {'new': [], 'old': []}
    last = {}
    for rnd in range(3):
        for tag, lib in (('new', 'libctclip_hip.so'), ('old', 'libctclip_hip_old.so')):
            out = f'/tmp/vq_ab_{tag}.pt'
            env = dict(os.environ, CTCLIP_HIP_LIB=os.path.join(LIBDIR, lib))
            subprocess.run([sys.executable, '-u', __file__, out], env=env, check=True)
            d = torch.load(out, weights_only=True)
            res[tag].append(d['ms'])
            last[tag] = d
    for tag in res:
        print(f'{tag}: median {statistics.median(res[tag]):.4f} ms  rounds {["%.4f" % v for v in res[tag]]}')
    print('candidates bit-identical:', torch.equal(last['new']['cand'], last['old']['cand']),
          ' second-best bit-identical:', torch.equal(last['new']['cand2'], last['old']['cand2']))


if __name__ == '__main__':
    main()
