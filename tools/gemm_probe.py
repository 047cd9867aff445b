"""Main-loop efficiency probe for the large-tile GEMM variants: 4096 x 4096 (256 tiles of 256^2,
one per CU) NT GEMM over K = 512..8192, bf16 out.  Run twice, with and without
CTCLIP_G256_DEBUG=1 (skip epilogue), to split the per-K-step cost from the fixed cost."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'ctpa-clip_amd'))
import torch  # noqa: E402

from ctclip_mi355x import kernels as K, _lib  # noqa: E402
from gemm_bench import timeit  # noqa: E402

torch.manual_seed(0)
M = N = int(os.environ.get('PROBE_MN', '4096'))
variants = [int(v) for v in os.environ.get('GEMM_VARIANTS', '8,1').split(',')]
for Kd in (512, 1024, 2048, 4096, 8192):
    x = (torch.rand(M, Kd, device='cuda') * 2 - 1).bfloat16()
    w = (torch.rand(N, Kd, device='cuda') * 2 - 1).bfloat16()
    out = torch.empty(M, N, device='cuda', dtype=torch.bfloat16)
    row = []
    for v in variants:
        _lib.lib().ctclip_gemm_set_variant(v)
        ms = timeit(lambda: K.linear(x, w, out=out), n=30)
        row.append(f'v{v} {ms * 1e3:8.1f} us {2 * M * N * Kd / ms / 1e9:7.1f} TF/s')
    lib_ms = timeit(lambda: torch.matmul(x, w.t()), n=30)
    row.append(f'lib {lib_ms * 1e3:8.1f} us {2 * M * N * Kd / lib_ms / 1e9:7.1f} TF/s')
    print(f'K={Kd:5d} ' + ' | '.join(row), flush=True)
