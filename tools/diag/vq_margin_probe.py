import os, sys
sys.path.insert(0, os.path.join(os.environ.get('GRAFT_REPO_ROOT', '.'), 'ctpa-clip_amd'))
sys.path.insert(0, os.path.join(os.environ.get('GRAFT_REPO_ROOT', '.'), 'tools'))
import torch
from ctclip_mi355x import kernels as K
from gemm_bench import timeit
torch.manual_seed(0)
M, D, C = 110592, 512, 8192
zf = torch.randn(M, D, device='cuda')
cb = torch.nn.functional.normalize(torch.randn(C, D, device='cuda'), dim=-1)
zb = zf.bfloat16()
cbb = cb.bfloat16()
xn_b = K.l2norm_scale_fwd(zb, 1, D, torch.ones(D, device='cuda'))
nt = C // 64
cand = torch.empty(M, nt, 2, device='cuda'); cand2 = torch.empty(M, nt, device='cuda')
K.gemm_raw(M, C, D, xn_b, D, True, cbb, D, True, cand, nt, C2=cand2, ldc2=nt, act=K.ACT_ARGMAX)
for mg in (2e-2, 8e-3, 4e-3):
    ms = timeit(lambda: K.vq_select(cand, zf, cb, margin=mg, want_xn=True, cand2=cand2))
    print(f'margin {mg:.0e}: vq_select {ms*1e3:.1f} us', flush=True)
