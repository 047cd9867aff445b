"""Thin, typed wrappers over the C-ABI (no autograd here).  Every function launches on
torch's current HIP stream and returns torch tensors allocated by the caching allocator."""
from __future__ import annotations

import torch

from . import _lib
from ._lib import GemmArgs, call, ptr, stream_ptr

BF16 = torch.bfloat16
F32 = torch.float32

ACT_NONE, ACT_GELU, ACT_GEGLU, ACT_ARGMAX = 0, 1, 2, 3


def _chk(t, name, dtype=None):
    if not t.is_cuda:
        raise ValueError(f'{name}: expected a device tensor')
    if dtype is not None and t.dtype != dtype:
        raise ValueError(f'{name}: expected {dtype}, got {t.dtype}')


def gemm_raw(M, N, K, A, lda, a_kcontig, B, ldb, b_kcontig, C, ldc, *, C2=None, ldc2=0, bias=None,
             R=None, ldr=0, alpha=1.0, act=ACT_NONE, accumulate=False, split_k=1, batch=1,
             sA=0, sB=0, sC=0, sC2=0, sR=0):
    a = GemmArgs()
    a.M, a.N, a.K = M, N, K
    a.A, a.lda, a.a_kcontig = ptr(A), lda, int(a_kcontig)
    a.B, a.ldb, a.b_kcontig = ptr(B), ldb, int(b_kcontig)
    a.C, a.ldc, a.c_f32 = ptr(C), ldc, int(C.dtype == F32)
    a.C2, a.ldc2 = ptr(C2), ldc2
    a.bias = ptr(bias)
    a.R, a.ldr, a.r_f32 = ptr(R), ldr, int(R is not None and R.dtype == F32)
    a.alpha, a.act, a.accumulate, a.split_k, a.batch = alpha, act, int(accumulate), split_k, batch
    a.sA, a.sB, a.sC, a.sC2, a.sR = sA, sB, sC, sC2, sR
    call('ctclip_gemm', _lib.ctypes.byref(a), stream_ptr())


def linear(x, w, *, bias=None, residual=None, out=None, out_dtype=BF16, act=ACT_NONE, out2=None, alpha=1.0,
           accumulate=False):
    """y[M,N] = x[M,K] @ w[N,K]^T (+bias) (+residual); x, w bf16 row-major."""
    M, K = x.shape
    N = w.shape[0]
    assert w.shape[1] == K and x.stride(1) == 1 and w.stride(1) == 1
    if out is None:
        out = torch.empty(M, N, device=x.device, dtype=out_dtype)
    gemm_raw(M, N, K, x, x.stride(0), True, w, w.stride(0), True, out, out.stride(0),
             C2=out2, ldc2=out2.stride(0) if out2 is not None else 0, bias=bias, R=residual,
             ldr=residual.stride(0) if residual is not None else 0, alpha=alpha, act=act, accumulate=accumulate)
    return out


def matmul_nn(dy, w, *, out=None, out_dtype=BF16, residual=None, accumulate=False, alpha=1.0):
    """dx[M,K] = dy[M,N] @ w[N,K] (w row-major, i.e. the nn.Linear weight)."""
    M, N = dy.shape
    K = w.shape[1]
    assert w.shape[0] == N
    if out is None:
        out = torch.empty(M, K, device=dy.device, dtype=out_dtype)
    gemm_raw(M, K, N, dy, dy.stride(0), True, w, w.stride(0), False, out, out.stride(0), R=residual,
             ldr=residual.stride(0) if residual is not None else 0, accumulate=accumulate, alpha=alpha)
    return out


def split_for(m_rows, tiles):
    """split-K factor for a dW GEMM whose reduction runs over m_rows tokens."""
    target = 512
    s = max(1, min(target // max(tiles, 1), m_rows // 1024))
    return max(1, s)


def matmul_tn(dy, x, *, out=None, accumulate=False, split_k=None, alpha=1.0):
    """dW[N,K] (f32) = dy[M,N]^T @ x[M,K]; reduction over the M tokens (split-K slabs)."""
    M, N = dy.shape
    K = x.shape[1]
    assert x.shape[0] == M
    if out is None:
        out = torch.zeros(N, K, device=dy.device, dtype=F32) if accumulate else \
            torch.empty(N, K, device=dy.device, dtype=F32)
    tiles = ((N + 127) // 128) * ((K + 127) // 128)
    s = split_for(M, tiles) if split_k is None else split_k
    if s <= 1:
        gemm_raw(N, K, M, dy, dy.stride(0), False, x, x.stride(0), False, out, out.stride(0),
                 accumulate=accumulate, alpha=alpha)
        return out
    slabs = torch.empty(s, N, K, device=dy.device, dtype=F32)
    gemm_raw(N, K, M, dy, dy.stride(0), False, x, x.stride(0), False, slabs, K, split_k=s, alpha=alpha)
    reduce_slabs(slabs, out, accumulate=accumulate)
    return out


def reduce_slabs(slabs, out, accumulate=False):
    s, rows, cols = slabs.shape
    call('ctclip_reduce_slabs', ptr(slabs), s, rows, cols, cols, ptr(out), out.stride(0),
         int(out.dtype == F32), int(accumulate), stream_ptr())
    return out
