"""Thin, typed wrappers over the C-ABI (no autograd here).  Every function launches on
torch's current HIP stream and returns torch tensors allocated by the caching allocator."""
from __future__ import annotations

import os

import torch

from . import _lib
from ._lib import GemmArgs, LnEpilogueArgs, call, ptr, stream_ptr

BF16 = torch.bfloat16
F32 = torch.float32
F16 = torch.float16

ACT_NONE, ACT_GELU, ACT_GEGLU, ACT_ARGMAX, ACT_GEGLU_BWD, ACT_L2N, ACT_GELU_BWD = 0, 1, 2, 3, 4, 5, 6


def _chk(t, name, dtype=None):
    if not t.is_cuda:
        raise ValueError(f'{name}: expected a device tensor')
    if dtype is not None and t.dtype != dtype:
        raise ValueError(f'{name}: expected {dtype}, got {t.dtype}')


class KernelTimer:
    """Optional HIP-event bracketing of tagged launches (bench.py's live roofline measurement).
    Events are recorded on torch's current stream — the stream the kernels launch on."""

    def __init__(self):
        self.active = False
        self.tags = set()
        self.events = []      # (tag, start, end, flops)

    def start(self, tags):
        self.active, self.tags, self.events = True, set(tags), []

    def stop(self):
        self.active = False

    def __call__(self, tag, flops):
        if not (self.active and tag in self.tags):
            return None
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        self.events.append((tag, s, e, flops))
        return e

    def summary(self, tag):
        torch.cuda.synchronize()
        ev = [(s, e, f) for t, s, e, f in self.events if t == tag]
        if not ev:
            return None
        ms = [s.elapsed_time(e) for s, e, _ in ev]
        return dict(launches=len(ev), avg_ms=sum(ms) / len(ms), flops=ev[0][2], total_ms=sum(ms),
                    total_flops=sum(f for _, _, f in ev))


TIMER = KernelTimer()


def gemm_raw(M, N, K, A, lda, a_kcontig, B, ldb, b_kcontig, C, ldc, *, C2=None, ldc2=0, bias=None,
             R=None, ldr=0, alpha=1.0, act=ACT_NONE, accumulate=False, split_k=1, batch=1,
             sA=0, sB=0, sC=0, sC2=0, sR=0, tag=None, flops=None, n2=0, B2=None, drop=None):
    end = TIMER(tag, flops if flops is not None else 2.0 * M * N * K * batch) if tag else None
    _gemm_raw(M, N, K, A, lda, a_kcontig, B, ldb, b_kcontig, C, ldc, C2=C2, ldc2=ldc2, bias=bias, R=R, ldr=ldr,
              alpha=alpha, act=act, accumulate=accumulate, split_k=split_k, batch=batch, sA=sA, sB=sB, sC=sC,
              sC2=sC2, sR=sR, n2=n2, B2=B2, drop=drop)
    if end is not None:
        end.record()


def _gemm_raw(M, N, K, A, lda, a_kcontig, B, ldb, b_kcontig, C, ldc, *, C2=None, ldc2=0, bias=None,
              R=None, ldr=0, alpha=1.0, act=ACT_NONE, accumulate=False, split_k=1, batch=1,
              sA=0, sB=0, sC=0, sC2=0, sR=0, n2=0, B2=None, drop=None):
    """drop = (p, seed): BERT hidden dropout on (A.B + bias) before the residual R (f32 C, act 0)."""
    if B2 is not None:
        assert B2.dtype == B.dtype and B2.shape == B.shape and B2.stride() == B.stride()
    h16 = A.dtype == F16       # fp16 operands (the 3D-ViT forward GEMMs): both, no split-K
    assert B.dtype == A.dtype, (A.dtype, B.dtype)
    s = 1 if h16 else _auto_split(M, N, K, act, split_k, batch, accumulate, C)
    if drop is not None:
        assert act == ACT_NONE and not accumulate and C.dtype == F32 and batch == 1 and ldc == N
        if s <= 1:     # no split-K combine to fold it into: GEMM (+ bias), then the dropout kernel
            _gemm_raw(M, N, K, A, lda, a_kcontig, B, ldb, b_kcontig, C, ldc, bias=bias, alpha=alpha, B2=B2)
            call('ctclip_dropout', ptr(C), ptr(R), ptr(C), ptr(C2), M * N, float(drop[0]),
                 int(drop[1]) & (2 ** 64 - 1), stream_ptr())
            return
        slabs = torch.empty(s, M, N, device=C.device, dtype=F32)
        _gemm_raw(M, N, K, A, lda, a_kcontig, B, ldb, b_kcontig, slabs, N, alpha=alpha, split_k=s, B2=B2)
        a = GemmArgs()
        a.C, a.ldc, a.c_f32 = ptr(C), ldc, 1
        a.C2, a.ldc2 = ptr(C2), ldc2
        a.bias = ptr(bias)
        a.R, a.ldr, a.r_f32 = ptr(R), ldr, int(R is not None and R.dtype == F32)
        call('ctclip_reduce_slabs_ep_drop', ptr(slabs), s, M, N, N, _lib.ctypes.byref(a), float(drop[0]),
             int(drop[1]) & (2 ** 64 - 1), stream_ptr())
        return
    if s > 1:
        # skinny GEMM (text tower, M = B * L tokens): split K into f32 slabs over ~4x more
        # workgroups than output tiles, then combine with the epilogue in one pass
        slabs = torch.empty(s, M, N, device=C.device, dtype=F32)
        _gemm_raw(M, N, K, A, lda, a_kcontig, B, ldb, b_kcontig, slabs, N, alpha=alpha, split_k=s, B2=B2)
        a = GemmArgs()
        a.C, a.ldc, a.c_f32 = ptr(C), ldc, int(C.dtype == F32)
        a.C2, a.ldc2 = ptr(C2), ldc2
        a.bias = ptr(bias)
        a.R, a.ldr, a.r_f32 = ptr(R), ldr, int(R is not None and R.dtype == F32)
        a.act, a.accumulate = act, int(accumulate)
        call('ctclip_reduce_slabs_ep', ptr(slabs), s, M, N, N, _lib.ctypes.byref(a), stream_ptr())
        return
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
    a.n2 = n2
    a.B2 = ptr(B2)
    a.ab_f16 = int(h16)
    a.r_f16 = int(R is not None and R.dtype == F16)
    call('ctclip_gemm', _lib.ctypes.byref(a), stream_ptr())


def _auto_split(M, N, K, act, split_k, batch, accumulate, C):
    """split-K factor for an epilogue GEMM that fills too few CUs with 128 x 128 tiles."""
    if split_k != 1 or batch != 1 or act not in (ACT_NONE, ACT_GELU) or K < 512 or N % 8 or C.stride(-1) != 1:
        return 1
    tiles = ((M + 127) // 128) * ((N + 127) // 128)
    if tiles >= 128 or M * N > (1 << 22):
        return 1
    return max(1, min(256 // tiles, K // 256))


def linear(x, w, *, bias=None, residual=None, out=None, out_dtype=BF16, act=ACT_NONE, out2=None, alpha=1.0,
           accumulate=False, tag=None, flops=None, l2n_scale=None, l2n_cols=0, w_lo=None, dropout=None,
           discard_out=False):
    """y[M,N] = x[M,K] @ w[N,K]^T (+bias) (+residual); x, w bf16 row-major.  l2n_scale (the [32]
    head-dim scale): out2[:, :l2n_cols] = per 32-column head l2norm(y) * scale, fused (act 5).
    w_lo: the bf16 lo image of a split f32 weight (cast_bf16_split): y = x @ (w + w_lo)^T.
    discard_out (fp16 GEGLU only): h is not stored, only out2 = g (the eval forward); returns None."""
    M, K = x.shape
    N = w.shape[0]
    assert w.shape[1] == K and x.stride(1) == 1 and w.stride(1) == 1
    if discard_out:
        assert act == ACT_GEGLU and x.dtype == F16 and out2 is not None and out is None
        a = GemmArgs()
        a.M, a.N, a.K = M, N, K
        a.A, a.lda, a.a_kcontig = ptr(x), x.stride(0), 1
        a.B, a.ldb, a.b_kcontig = ptr(w), w.stride(0), 1
        a.C, a.ldc = None, N
        a.C2, a.ldc2 = ptr(out2), out2.stride(0)
        a.alpha, a.act, a.split_k, a.batch, a.ab_f16 = alpha, ACT_GEGLU, 1, 1, 1
        end = TIMER(tag, flops if flops is not None else 2.0 * M * N * K) if tag else None
        call('ctclip_gemm', _lib.ctypes.byref(a), stream_ptr())
        if end is not None:
            end.record()
        return None
    if out is None:
        out = torch.empty(M, N, device=x.device, dtype=out_dtype)
    if l2n_scale is not None:
        assert bias is None and residual is None and out2 is not None and l2n_scale.numel() == 32
        assert l2n_scale.dtype == torch.float32 and l2n_scale.is_contiguous()
        act, bias = ACT_L2N, l2n_scale
    gemm_raw(M, N, K, x, x.stride(0), True, w, w.stride(0), True, out, out.stride(0),
             C2=out2, ldc2=out2.stride(0) if out2 is not None else 0, bias=bias, R=residual,
             ldr=residual.stride(0) if residual is not None else 0, alpha=alpha, act=act, accumulate=accumulate,
             tag=tag, flops=flops, n2=l2n_cols, B2=w_lo, drop=dropout)
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


# ------------------------------------------- LayerNorm fused into N = 512 GEMM epilogues
# ctclip_gemm_ln: the two 256-column tiles of a row block exchange per-row statistics inside the
# launch through a per-stream buffer of {epoch, value} granules (zeroed once; every launch uses a
# fresh epoch, so nothing needs clearing between launches).  CTCLIP_LN_FUSED=0: the GEMM and the
# LayerNorm kernel run separately (A/B switch).
LN_FUSED = os.environ.get('CTCLIP_LN_FUSED', '1') != '0'
# the backward form (GEMM + LayerNorm backward + residual) measured SLOWER than the pair it
# replaces (profiles/r03o_ln_bench.log: 510 vs 476 us at K = 2,816, 265 vs 226 us at K = 256; the
# stand-alone LayerNorm backward streams at ~6 TB/s, the fused epilogue at 8 waves per CU does not),
# so it is opt-in; the forward form is the default (171 vs 192 us)
LN_FUSED_BWD = os.environ.get('CTCLIP_LN_FUSED_BWD', '0') != '0'
_XCHG = {}       # (device, stream) -> [int64 buffer, last epoch]
_LN_STATUS = {}  # device -> int32[1], set by a launch whose partner statistics never arrived
_CT_EINVAL, _CT_ESHAPE = 1001, 1003
_PEG_BWD_X32 = os.environ.get('CTCLIP_PEG_BWD_X32', '1') != '0'
# Fail loud: the exchange's partner wait is bounded, and a launch that gives up leaves
# wrong LayerNorm outputs and sets the device status word.  The fused form is therefore only used
# where something reads that word every step: inside ``ln_guard()`` (trainer.CTClipTrainer wraps
# its forward / backward in it, passes the word to the Adam kernel as its skip guard -- a step with
# a timed-out exchange is never applied -- and raises ``LayerNormExchangeError`` on the host, at
# the latest two steps later, or in ``check()`` / ``flush()``).  Elsewhere the GEMM and the
# LayerNorm kernel run separately.
_LN_GUARD = [0]
_LN_DEBUG = {'skip_publish': 0, 'spin_limit': 0}


class _LnGuard:
    def __enter__(self):
        _LN_GUARD[0] += 1
        return self

    def __exit__(self, *exc):
        _LN_GUARD[0] -= 1
        return False


def ln_guard():
    """Context in which the model may use the LayerNorm-fused GEMMs: the caller promises to read
    ``ln_status_tensor`` (trainer.CTClipTrainer does, every step)."""
    return _LnGuard()


def ln_guarded():
    return _LN_GUARD[0] > 0


def set_ln_debug(skip_publish=False, spin_limit=0):
    """Test knob: tile 1 of row block 0 never publishes its statistics (its partner times out after
    ``spin_limit`` polls, 0 = the library default ~0.1 s).  Returns the previous setting."""
    old = dict(_LN_DEBUG)
    _LN_DEBUG['skip_publish'], _LN_DEBUG['spin_limit'] = int(bool(skip_publish)), int(spin_limit)
    return old


def _xchg(M, device):
    st = torch.cuda.current_stream(device)
    key = (device.index, st.cuda_stream)
    e = _XCHG.get(key)
    if e is None or e[0].numel() < 4 * M:
        e = _XCHG[key] = [torch.zeros(4 * M, dtype=torch.int64, device=device), 0]
    if e[1] >= 0xFFFFFFFF:        # epochs exhausted: clear the granules (stream-ordered) and restart
        e[0].zero_()
        e[1] = 0
    e[1] += 1
    return e[0], e[1]


def ln_status_tensor(device):
    """The device's sticky int32[1] status word of the LayerNorm-fused GEMMs (created zeroed)."""
    device = torch.device(device)
    idx = device.index if device.index is not None else torch.cuda.current_device()
    s = _LN_STATUS.get(idx)
    if s is None:
        s = _LN_STATUS[idx] = torch.zeros(1, dtype=torch.int32, device=torch.device('cuda', idx))
    return s


_ln_status = ln_status_tensor


def reset_ln_status(device=None):
    """Clear the status word (after handling a LayerNormExchangeError)."""
    ln_status_tensor(device or torch.device('cuda', torch.cuda.current_device())).zero_()


def ln_fused_status(device=None):
    """1 if any LayerNorm-fused GEMM on `device` gave up waiting for its partner tile (then its
    outputs are wrong); 0 otherwise.  Synchronises."""
    s = _LN_STATUS.get((device or torch.device('cuda', torch.cuda.current_device())).index)
    return 0 if s is None else int(s.item())


def ln_fusable(M, N, bwd=False):
    return LN_FUSED and (LN_FUSED_BWD or not bwd) and N == 512 and M > 0 and M % 2048 == 0


def _gemm_ln(M, K, A, B, b_kcontig, C, C2, R, ln, tag=None, flops=None):
    """Returns False (nothing launched) when the library refuses the configuration."""
    assert A.dtype == B.dtype
    a = GemmArgs()
    a.ab_f16 = int(A.dtype == F16)
    a.M, a.N, a.K = M, 512, K
    a.A, a.lda, a.a_kcontig = ptr(A), A.stride(0), 1
    a.B, a.ldb, a.b_kcontig = ptr(B), B.stride(0), int(b_kcontig)
    a.C, a.ldc, a.c_f32 = ptr(C), C.stride(0), 1
    a.C2, a.ldc2 = ptr(C2), C2.stride(0) if C2 is not None else 0
    a.R, a.ldr, a.r_f32 = ptr(R), R.stride(0) if R is not None else 0, 1
    a.alpha, a.act, a.accumulate, a.split_k, a.batch = 1.0, 0, 0, 1, 1
    xb, ep = _xchg(M, A.device)
    ln.xchg, ln.epoch = ptr(xb), ep
    ln.status = ptr(_ln_status(A.device))
    ln.spin_limit, ln.debug = _LN_DEBUG['spin_limit'], _LN_DEBUG['skip_publish']
    end = TIMER(tag, flops if flops is not None else 2.0 * M * 512 * K) if tag else None
    rc = _lib.lib().ctclip_gemm_ln(_lib.ctypes.byref(a), _lib.ctypes.byref(ln), stream_ptr())
    if rc in (_CT_EINVAL, _CT_ESHAPE):
        return False
    if rc != 0:
        raise _lib.KernelError(f'ctclip_gemm_ln failed: {rc}')
    if end is not None:
        end.record()
    return True


def linear_residual_ln(x, w, residual, gamma, beta, eps, *, tag=None, y16=False, eval_only=False):
    """x1 = residual + x @ w^T (w [512, K] nn.Linear weight) and y = LayerNorm(x1) (gamma, beta;
    bf16) in ONE launch (ctclip_gemm_ln mode 1).  Returns (x1 f32, x1 bf16, y bf16, mean, rstd) --
    plus y's fp16 copy when y16 -- or None when the shape / configuration does not allow the fused
    form.  x, w fp16: the fp16 GEMM.  eval_only (with y16): the backward-only bf16 x1 and y are not
    written (None)."""
    M, K = x.shape
    if not ln_fusable(M, w.shape[0]) or K % 64 or residual.dtype != F32:
        return None
    assert y16 or not eval_only
    dev = x.device
    x1f = torch.empty(M, 512, device=dev, dtype=F32)
    x1b = None if eval_only else torch.empty(M, 512, device=dev, dtype=BF16)
    y = None if eval_only else torch.empty(M, 512, device=dev, dtype=BF16)
    mean = torch.empty(M, device=dev, dtype=F32)
    rstd = torch.empty(M, device=dev, dtype=F32)
    ln = LnEpilogueArgs()
    ln.mode, ln.gamma, ln.beta, ln.eps = 1, ptr(gamma), ptr(beta), eps
    ln.Y, ln.ldy, ln.mean, ln.rstd = ptr(y), 512, ptr(mean), ptr(rstd)
    yh = torch.empty(M, 512, device=dev, dtype=F16) if y16 else None
    ln.Y16 = ptr(yh)
    if not _gemm_ln(M, K, x, w, True, x1f, x1b, residual, ln, tag=tag):
        return None
    if y16:
        return x1f, x1b, y, mean, rstd, yh
    return x1f, x1b, y, mean, rstd


def matmul_nn_ln_bwd(dy, w, x, mean, rstd, gamma, dres, *, dgamma_out, dbeta_out=None):
    """dx = LayerNorm'(dy @ w) + dres in ONE launch (ctclip_gemm_ln mode 2): dy [M, N] bf16,
    w [N, 512] (the nn.Linear weight whose input was LayerNorm(x)), x [M, 512] bf16 with the
    forward's mean / rstd; the gamma / beta gradients accumulate into dgamma_out / dbeta_out
    (deferred partial reductions).  Returns (dx f32, dx bf16), or None when not fusable."""
    M, N = dy.shape
    if not (LN_FUSED_BWD and ln_fusable(M, w.shape[1])) or N % 64 or dres is None or dres.dtype != F32:
        return None
    dev = dy.device
    dxf = torch.empty(M, 512, device=dev, dtype=F32)
    dxb = torch.empty(M, 512, device=dev, dtype=BF16)
    nb = M // 128
    pg = torch.empty(nb, 512, device=dev, dtype=F32)
    pb = torch.empty(nb, 512, device=dev, dtype=F32) if dbeta_out is not None else None
    ln = LnEpilogueArgs()
    ln.mode, ln.gamma, ln.beta, ln.eps = 2, ptr(gamma), None, 0.0
    ln.mean, ln.rstd, ln.X, ln.ldx = ptr(mean), ptr(rstd), ptr(x), x.stride(0)
    ln.part_gamma, ln.part_beta = ptr(pg), ptr(pb)
    if not _gemm_ln(M, N, dy, w, False, dxf, dxb, dres, ln):
        return None
    reduce_param_partials(pg, dgamma_out, True)
    if dbeta_out is not None:
        reduce_param_partials(pb, dbeta_out, True)
    return dxf, dxb


def matmul_nn_gelu_bwd(dy, w, pre, out=None):
    """dx = (dy @ w) * gelu'(pre) in one GEMM (act 6): dy [M, N] bf16, w [N, K] (the nn.Linear
    weight), pre [M, K] bf16 (the act-1 pre-activation); returns dx [M, K] bf16."""
    M, N = dy.shape
    K = w.shape[1]
    assert w.shape[0] == N and pre.shape == (M, K) and pre.dtype == BF16
    if out is None:
        out = torch.empty(M, K, device=dy.device, dtype=BF16)
    gemm_raw(M, K, N, dy, dy.stride(0), True, w, w.stride(0), False, out, out.stride(0), R=pre, ldr=pre.stride(0),
             act=ACT_GELU_BWD)
    return out


def split_for(m_rows, tiles):
    """split-K factor for a dW GEMM whose reduction runs over m_rows tokens."""
    target = 512
    s = max(1, min(target // max(tiles, 1), m_rows // 1024))
    return max(1, s)


def matmul_tn(dy, x, *, out=None, accumulate=False, split_k=None, alpha=1.0, tag=None, flops=None, unpack=None):
    """dW[N,K] (f32) = dy[M,N]^T @ x[M,K]; reduction over the M tokens (split-K slabs).
    tag / flops: KernelTimer bracketing of the GEMM launch (not the slab reduction).
    unpack=(dst, rowmap, cols): accumulate dW[r, :cols] into dst[rowmap[r]] (rowmap None = identity,
    negative entries dropped) instead of returning dW -- with split-K slabs in one reduction pass
    (ctclip_reduce_slabs_rows), bit-identical to dW followed by unpack_rows."""
    M, N = dy.shape
    K = x.shape[1]
    assert x.shape[0] == M
    if out is None:
        out = torch.zeros(N, K, device=dy.device, dtype=F32) if accumulate else \
            torch.empty(N, K, device=dy.device, dtype=F32)
    if split_k is not None:
        s = split_k
    elif N >= 256 and K >= 256 and M % 64 == 0 and M >= 64 * 1024:
        # 8-phase 256x256x64 kernel (gemm256.hip): one wave of <= 256 workgroups (one per CU),
        # each reducing a long K-chunk; the slabs are summed by reduce_slabs
        t256 = ((N + 255) // 256) * ((K + 255) // 256)
        s = max(1, 256 // t256)
        if t256 * s < 160:
            s = split_for(M, ((N + 127) // 128) * ((K + 127) // 128))
    else:
        s = split_for(M, ((N + 127) // 128) * ((K + 127) // 128))
    if s <= 1:
        gemm_raw(N, K, M, dy, dy.stride(0), False, x, x.stride(0), False, out, out.stride(0),
                 accumulate=accumulate, alpha=alpha, tag=tag, flops=flops)
        if unpack is not None:
            dst, rowmap, cols = unpack
            return unpack_rows(out, dst, rowmap=rowmap, cols=cols, accumulate=True)
        return out
    slabs = torch.empty(s, N, K, device=dy.device, dtype=F32)
    gemm_raw(N, K, M, dy, dy.stride(0), False, x, x.stride(0), False, slabs, K, split_k=s, alpha=alpha, tag=tag,
             flops=flops)
    if unpack is not None:
        dst, rowmap, cols = unpack
        assert dst.dtype == F32 and dst.stride(1) == 1 and cols <= K
        assert rowmap is None or (rowmap.dtype == torch.int32 and rowmap.numel() == N)
        call('ctclip_reduce_slabs_rows', ptr(slabs), s, N, cols, K, ptr(rowmap), ptr(dst), dst.stride(0), 1,
             stream_ptr())
        return dst
    reduce_slabs(slabs, out, accumulate=accumulate)
    return out


def reduce_slabs(slabs, out, accumulate=False):
    s, rows, cols = slabs.shape
    call('ctclip_reduce_slabs', ptr(slabs), s, rows, cols, cols, ptr(out), out.stride(0),
         int(out.dtype == F32), int(accumulate), stream_ptr())
    return out


# ------------------------------------------------- deferred parameter-gradient reductions
# The LN / l2norm / bias backward kernels leave per-block partials [nb][D] of a parameter
# gradient; each used to be summed into .grad by its own ~10 us launch (72 per step on the image
# tower's stream).  Inside a backward pass they are queued per stream instead and summed by ONE
# batched launch (ctclip_reduce_slabs_multi, bit-identical to the single reduction) when the pass
# ends (autograd callback), or earlier when a gradient bucket's all-reduce is about to read them
# (dist_sync.BucketedGradSync).  CTCLIP_DEFER_REDUCE=0 restores the immediate launches.
DEFER_REDUCE = os.environ.get('CTCLIP_DEFER_REDUCE', '1') != '0'
_DEFERRED = {}        # stream id -> (stream, [(slabs, out, accumulate), ...])
_CB_QUEUED = [None]   # graph task id whose end-of-pass callback is queued (None: none)


def _graph_task():
    try:
        return torch._C._current_graph_task_id()
    except AttributeError:
        return -1


def _in_backward():
    return _graph_task() != -1


def discard_deferred():
    """Drop every queued reduction and forget the queued callback: the exception path of a
    backward pass (trainer.forward_backward) -- a pass that raised never runs its callback, and
    its partial sums must not land in the next pass's gradients."""
    _DEFERRED.clear()
    _CB_QUEUED[0] = None


def flush_reductions(lo=None, hi=None):
    """Launch the queued reductions (each on the stream that queued it), all of them or only those
    whose output lies in the byte range [lo, hi) (a gradient bucket); returns the streams used."""
    used = []
    for k in list(_DEFERRED):
        st, jobs = _DEFERRED[k]
        if lo is None:
            take, keep = jobs, []
        else:
            take = [j for j in jobs if lo <= j[1].data_ptr() < hi]
            keep = [j for j in jobs if not (lo <= j[1].data_ptr() < hi)]
        if keep:
            _DEFERRED[k] = (st, keep)
        else:
            del _DEFERRED[k]
        if not take:
            continue
        # the jobs of one launch run concurrently and each read-add-writes its output: jobs that
        # share an output (a parameter used twice in one pass) go to successive launches, in
        # queue order, so no update is lost
        while take:
            seen, batch, rest = set(), [], []
            for j in take:
                (rest if j[1].data_ptr() in seen else batch).append(j)
                seen.add(j[1].data_ptr())
            arr = (_lib.SlabJob * len(batch))()
            for i, (sl, out, acc) in enumerate(batch):
                arr[i].slabs, arr[i].nslab, arr[i].cols = sl.data_ptr(), sl.shape[0], sl.shape[-1]
                arr[i].out, arr[i].accumulate = out.data_ptr(), int(acc)
            call('ctclip_reduce_slabs_multi', arr, len(batch), st.cuda_stream)
            take = rest
        # the partial buffers were allocated on `st`; freeing them after this launch is ordered
        used.append(st)
    return used


def _end_of_backward():
    _CB_QUEUED[0] = None
    flush_reductions()


def reduce_param_partials(part, out, accumulate):
    """out[D] (+)= sum of part[nb][D]: deferred inside a backward pass (see above)."""
    nb, D = part.shape[0], part.shape[-1]
    if (DEFER_REDUCE and nb >= 16 and out.dtype == F32 and out.is_contiguous() and part.is_contiguous()
            and D % 4 == 0 and _in_backward()):
        st = torch.cuda.current_stream(part.device)
        _DEFERRED.setdefault(st.cuda_stream, (st, []))[1].append((part, out.view(-1), accumulate))
        task = _graph_task()
        if _CB_QUEUED[0] != task:      # a new pass (or one whose predecessor raised before its end)
            torch.autograd.Variable._execution_engine.queue_callback(_end_of_backward)
            _CB_QUEUED[0] = task
        return out
    return reduce_slabs(part.view(nb, 1, D), out.view(1, D), accumulate=accumulate)


# ----------------------------------------------------------------------------- reductions
def nblocks_for(rows, cap=1024):
    """Workgroups of the LayerNorm backward (4 waves each; a wave walks its rows one at a time):
    >= 64 rows per workgroup on long inputs (the 3D-ViT's 110,592 tokens: the parameter-gradient
    partial slabs stay small), but one row per wave on short ones (BERT's 1,024 tokens: 256
    workgroups instead of 16, whose waves walked 16 rows one memory latency after another)."""
    if not _LNB_WIDE:
        return int(max(1, min(cap, (rows + 63) // 64)))
    return int(max(1, min(cap, max((rows + 63) // 64, min(256, (rows + 3) // 4)))))


_LNB_WIDE = os.environ.get('CTCLIP_LNB_WIDE', '1') != '0'   # A/B switch of nblocks_for's short-input rule
_LNB_CAP = int(os.environ.get('CTCLIP_LNB_CAP', '1024'))      # LayerNorm-backward workgroup cap (A/B)


def colsum(x, out=None, accumulate=False):
    """Column sums of x[rows, cols] (bf16 or f32) -> f32 [cols]."""
    rows, cols = x.shape
    nb = int(max(1, min(256, rows // 8)))   # >= 8 rows per block: short (text-tower) inputs fill the chip
    part = torch.empty(nb, cols, device=x.device, dtype=F32)
    call('ctclip_colsum', ptr(x), int(x.dtype == F32), x.stride(0), rows, cols, ptr(part), nb, stream_ptr())
    if out is None:
        out = torch.zeros(cols, device=x.device, dtype=F32) if accumulate else torch.empty(cols, device=x.device,
                                                                                           dtype=F32)
    if accumulate:
        reduce_param_partials(part, out, accumulate)
    else:
        reduce_slabs(part.view(nb, 1, cols), out.view(1, cols), accumulate=accumulate)
    return out


# ----------------------------------------------------------------------------- LayerNorm
def layernorm_fwd(x, gamma, beta, eps, *, out_bf16=True, out_f32=False, out_f16=False, out_x3=False):
    """Returns (y bf16, y f32, mean, rstd), plus y's fp16 copy when out_f16 (requires out_bf16), or
    its split-fp16 pair (hi, lo) when out_x3 (the x3 GEMM's A operand)."""
    rows, D = x.shape
    yb = torch.empty(rows, D, device=x.device, dtype=BF16) if out_bf16 else None
    yf = torch.empty(rows, D, device=x.device, dtype=F32) if out_f32 else None
    yh = torch.empty(rows, D, device=x.device, dtype=F16) if out_f16 or out_x3 else None
    yl = torch.empty(rows, D, device=x.device, dtype=F16) if out_x3 else None
    mean = torch.empty(rows, device=x.device, dtype=F32)
    rstd = torch.empty(rows, device=x.device, dtype=F32)
    call('ctclip_layernorm_fwd_x3', ptr(x), int(x.dtype == F32), x.stride(0), rows, D, ptr(gamma), ptr(beta), eps,
         ptr(yb), ptr(yh), ptr(yl), D, ptr(yf), D, ptr(mean), ptr(rstd),
         ptr(status_word(x.device)) if yh is not None else None, stream_ptr())
    if out_x3:
        return yb, yf, mean, rstd, (yh, yl)
    if out_f16:
        return yb, yf, mean, rstd, yh
    return yb, yf, mean, rstd


def layernorm_bwd(dy, x, mean, rstd, gamma, *, dres=None, want_beta=True, dx_f32=True, dx_bf16=True,
                  dgamma_out=None, dbeta_out=None):
    """Returns (dx_f32, dx_bf16, dgamma, dbeta).  dgamma_out / dbeta_out: accumulate the
    parameter gradients into these f32 tensors instead of returning fresh ones."""
    rows, D = x.shape
    nb = nblocks_for(rows, _LNB_CAP)
    dxf = torch.empty(rows, D, device=x.device, dtype=F32) if dx_f32 else None
    dxb = torch.empty(rows, D, device=x.device, dtype=BF16) if dx_bf16 else None
    pg = torch.empty(nb, D, device=x.device, dtype=F32)
    pb = torch.empty(nb, D, device=x.device, dtype=F32) if want_beta else None
    call('ctclip_layernorm_bwd', ptr(dy), int(dy.dtype == F32), dy.stride(0), ptr(x), int(x.dtype == F32),
         x.stride(0), ptr(mean), ptr(rstd), ptr(gamma), rows, D, ptr(dres),
         dres.stride(0) if dres is not None else 0, ptr(dxf), D, ptr(dxb), D, ptr(pg), ptr(pb), nb, stream_ptr())
    if dgamma_out is not None:      # a parameter's .grad: possibly deferred (reduce_param_partials)
        dg = reduce_param_partials(pg, dgamma_out, True)
    else:
        dg = torch.empty(D, device=x.device, dtype=F32)
        reduce_slabs(pg.view(nb, 1, D), dg.view(1, D))
    db = None
    if want_beta:
        if dbeta_out is not None:
            db = reduce_param_partials(pb, dbeta_out, True)
        else:
            db = torch.empty(D, device=x.device, dtype=F32)
            reduce_slabs(pb.view(nb, 1, D), db.view(1, D))
    return dxf, dxb, dg, db


def layernorm_bwd_drop(dy, x, mean, rstd, gamma, p, seed, *, dgamma_out, dbeta_out, dbias_out=None):
    """Backward of LN(dropout(dense) + res) (BERT, p > 0): returns (dx f32 = the residual
    branch's gradient, bf16(dropout(dx)) = the dense output's gradient); the LN gamma / beta
    gradients and, if given, the dense bias gradient (column sums of the bf16 output) accumulate
    into dgamma_out / dbeta_out / dbias_out (deferred partial reductions)."""
    rows, D = x.shape
    assert dy.dtype == F32 and x.dtype == F32
    nb = nblocks_for(rows, _LNB_CAP)
    dxf = torch.empty(rows, D, device=x.device, dtype=F32)
    dxb = torch.empty(rows, D, device=x.device, dtype=BF16)
    pg = torch.empty(nb, D, device=x.device, dtype=F32)
    pb = torch.empty(nb, D, device=x.device, dtype=F32)
    pd = torch.empty(nb, D, device=x.device, dtype=F32) if dbias_out is not None else None
    call('ctclip_layernorm_bwd_drop', ptr(dy), 1, dy.stride(0), ptr(x), 1, x.stride(0), ptr(mean), ptr(rstd),
         ptr(gamma), rows, D, ptr(dxf), D, ptr(dxb), D, ptr(pg), ptr(pb), ptr(pd), nb, float(p),
         int(seed) & (2 ** 64 - 1), stream_ptr())
    reduce_param_partials(pg, dgamma_out, True)
    reduce_param_partials(pb, dbeta_out, True)
    if dbias_out is not None:
        reduce_param_partials(pd, dbias_out, True)
    return dxf, dxb


def l2norm_scale_fwd(x, H, D, scale, out=None):
    rows = x.shape[0]
    if out is None:
        out = torch.empty(rows, H * D, device=x.device, dtype=BF16)
    call('ctclip_l2norm_scale_fwd', ptr(x), x.stride(0), rows, H, D, ptr(scale), ptr(out), out.stride(0),
         stream_ptr())
    return out


def l2norm_scale_bwd(x, dy, H, D, scale, out, ds_out=None):
    """dx into `out`; returns dscale (accumulated into ds_out when given)."""
    rows = x.shape[0]
    lpr = H * D // 8
    nb = 2048       # 8 workgroups per CU: the row loop is load-latency bound
    while (nb * 256) % lpr:
        nb += 1
    part = torch.empty(nb, D, device=x.device, dtype=F32)
    call('ctclip_l2norm_scale_bwd', ptr(x), x.stride(0), ptr(dy), dy.stride(0), rows, H, D, ptr(scale), ptr(out),
         out.stride(0), ptr(part), nb, stream_ptr())
    if ds_out is not None:
        return reduce_param_partials(part, ds_out, True)
    ds = torch.empty(D, device=x.device, dtype=F32)
    reduce_slabs(part.view(nb, 1, D), ds.view(1, D))
    return ds


# ----------------------------------------------------------------------------- elementwise
def matmul_nn_geglu_bwd(dy, w2p, h, out=None):
    """dh = geglu_bwd(dy @ w2p, h) in one GEMM (act 4): dy [M, D] bf16, w2p [D, G] (the padded
    FeedForward W2), h [M, 2G] bf16 the GEGLU pre-activation [x | gate] per 64-column group, or fp16
    in the derivative form [gelu(gate) | x gelu'(gate)] the fp16 FF1 writes (round 6); returns dh
    [M, 2G] bf16."""
    M, D = dy.shape
    G = w2p.shape[1]
    assert w2p.shape[0] == D and h.shape == (M, 2 * G)
    if out is None:
        out = torch.empty(M, 2 * G, device=dy.device, dtype=BF16)
    gemm_raw(M, G, D, dy, dy.stride(0), True, w2p, w2p.stride(0), False, out, out.stride(0), R=h, ldr=h.stride(0),
             act=ACT_GEGLU_BWD)
    return out


def geglu_bwd(dg, h, out=None):
    """Stand-alone GEGLU backward from the bf16 pre-activation h (an fp16 h is in the derivative form
    and goes through matmul_nn_geglu_bwd)."""
    assert h.dtype == BF16, h.dtype
    rows, gcols = dg.shape
    if out is None:
        out = torch.empty(rows, 2 * gcols, device=dg.device, dtype=BF16)
    call('ctclip_geglu_bwd', ptr(dg), dg.stride(0), ptr(h), h.stride(0), rows, gcols, ptr(out), out.stride(0),
         stream_ptr())
    return out


def gelu_bwd(dy, pre):
    out = torch.empty_like(pre)
    call('ctclip_gelu_bwd', ptr(dy), ptr(pre), ptr(out), pre.numel(), stream_ptr())
    return out


def pack_rows(src, rows_dst, cols_dst, rowmap=None, colscale=None, out=None):
    rows, cols = src.shape
    if out is None:
        out = torch.empty(rows_dst, cols_dst, device=src.device, dtype=BF16)
    call('ctclip_pack_rows', ptr(src), src.stride(0), ptr(rowmap), rows_dst, cols, cols_dst, ptr(colscale), ptr(out),
         out.stride(0), stream_ptr())
    return out


def pack_rows_h16(src, rows_dst, cols_dst, rowmap=None, colscale=None, out=None):
    """fp16 working weight (the fp16 forward GEMMs), as pack_rows."""
    rows, cols = src.shape
    if out is None:
        out = torch.empty(rows_dst, cols_dst, device=src.device, dtype=F16)
    call('ctclip_pack_rows_h16', ptr(src), src.stride(0), ptr(rowmap), rows_dst, cols, cols_dst, ptr(colscale),
         ptr(out), out.stride(0), stream_ptr())
    return out


def pack_rows_f32(src, rows_dst, cols_dst, rowmap=None, colscale=None, out=None):
    """f32 working weight: out[r][c] = src[rowmap[r]][c] * colscale[c] (zero padding), as pack_rows."""
    rows, cols = src.shape
    if out is None:
        out = torch.empty(rows_dst, cols_dst, device=src.device, dtype=F32)
    call('ctclip_pack_rows_f32', ptr(src), src.stride(0), ptr(rowmap), rows_dst, cols, cols_dst, ptr(colscale),
         ptr(out), out.stride(0), stream_ptr())
    return out


def unpack_rows(src, dst, rowmap=None, cols=None, accumulate=True):
    rows_src = src.shape[0]
    cols = dst.shape[1] if cols is None else cols
    call('ctclip_unpack_rows', ptr(src), src.stride(0), ptr(rowmap), rows_src, cols, ptr(dst), dst.stride(0),
         int(accumulate), stream_ptr())
    return dst


def cast_bf16(x, out=None):
    if out is None:
        out = torch.empty(x.shape, device=x.device, dtype=BF16)
    call('ctclip_cast_f32_bf16', ptr(x), ptr(out), x.numel(), stream_ptr())
    return out


def cast_bf16_split(x, hi=None, lo=None):
    """(hi, lo) = (bf16(x), bf16(x - hi)) of an f32 tensor: x to ~16 mantissa bits as two bf16 images."""
    if hi is None:
        hi = torch.empty(x.shape, device=x.device, dtype=BF16)
    if lo is None:
        lo = torch.empty(x.shape, device=x.device, dtype=BF16)
    call('ctclip_cast_f32_bf16_split', ptr(x), ptr(hi), ptr(lo), x.numel(), stream_ptr())
    return hi, lo


def add_f32(a, b, out=None, out_bf16=None):
    call('ctclip_add_f32', ptr(a), ptr(b), ptr(out), ptr(out_bf16), a.numel(), stream_ptr())


# ----------------------------------------------------------------------------- patch embed
def patch_ln(video, is_hu, PT, P, offs, eps=1e-5, ld=None, want_f16=False, want_x3=False, want_bf16=True):
    """LayerNorm'd patch rows [tokens, ld] bf16 (columns pd..ld-1 zero: K padding for the GEMM);
    with want_f16 also their fp16 copy (returns (bf16, f16)); with want_x3 their split-fp16 pair
    (returns (bf16, (hi, lo))).  want_bf16=False (with want_f16): the bf16 rows -- the weight
    gradient's operand -- are not written (None; the eval forward)."""
    B, C, Fr, H, W = video.shape
    T, Hg, Wg = Fr // PT, H // P, W // P
    pd = C * PT * P * P
    ld = pd if ld is None else ld
    out = torch.empty(B * T * Hg * Wg, ld, device=video.device, dtype=BF16) if want_bf16 else None
    out16 = torch.empty(B * T * Hg * Wg, ld, device=video.device, dtype=F16) if want_f16 or want_x3 else None
    out16lo = torch.empty(B * T * Hg * Wg, ld, device=video.device, dtype=F16) if want_x3 else None
    end = TIMER('patch_ln', 0.0)      # (bench.py: the patch LayerNorm's in-step duration)
    call('ctclip_patch_ln_x3', ptr(video), int(video.dtype == F32), int(is_hu), B, C, Fr, H, W, PT, P, ptr(offs), eps,
         ptr(out), ptr(out16), ptr(out16lo), ld, stream_ptr())
    if end is not None:
        end.record()
    if want_x3:
        return out, (out16, out16lo)
    return (out, out16) if want_f16 else out


def unpatch_mse(pix, video, is_hu, PT, P, offs, want_grad=True, want_recon=False):
    """(loss [1] f32, grad [tokens, pd] or None, recon (B,C,F,H,W) or None) of
    F.mse_loss(video, rearrange(pix)) -- the inverse patch map of patch_ln."""
    B, C, Fr, H, W = video.shape
    pd = C * PT * P * P
    n = pix.shape[0]
    grad = torch.empty(n, pd, device=pix.device, dtype=F32) if want_grad else None
    recon = torch.empty(B, C, Fr, H, W, device=pix.device, dtype=F32) if want_recon else None
    part = torch.empty(n, device=pix.device, dtype=F32)
    loss = torch.empty(1, device=pix.device, dtype=F32)
    call('ctclip_unpatch_mse', ptr(pix), pix.stride(0), ptr(video), int(video.dtype == F32), int(is_hu), B, C, Fr, H, W,
         PT, P, ptr(offs), ptr(grad), pd, ptr(recon), ptr(part), ptr(loss), stream_ptr())
    return loss, grad, recon


def patch_wgrad(G, cs, W, g, b, dW, dg, db, accumulate=True):
    N, K = G.shape
    call('ctclip_patch_wgrad', ptr(G), ptr(cs), ptr(W), ptr(g), ptr(b), N, K, ptr(dW), ptr(dg), ptr(db),
         int(accumulate), stream_ptr())


# ----------------------------------------------------------------------------- PEG
def peg_fwd(xb, xf, B, T, H, W, weight, bias, mode):
    D = xb.shape[1]
    outf = torch.empty_like(xf)
    outb = torch.empty_like(xb)
    call('ctclip_peg_fwd', ptr(xb), ptr(xf), B, T, H, W, D, ptr(weight), ptr(bias), mode, ptr(outf), ptr(outb),
         stream_ptr())
    return outf, outb


def peg_fwd_stats(xb, xf, B, T, H, W, weight, bias, mode, eps=1e-5):
    """peg_fwd plus the LayerNorm statistics of its output rows (the attention's pre-norm,
    ct_clip/attention.py:139-141): the conv kernel leaves (mean, M2) per 64-channel group and one
    light pass merges them.  Returns (out_f32, out_bf16, mean [M], rstd [M])."""
    M, D = xb.shape
    outf = torch.empty_like(xf)
    outb = torch.empty_like(xb)
    part = torch.empty(D // 64, M, 2, device=xb.device, dtype=F32)
    call('ctclip_peg_fwd_stats', ptr(xb), ptr(xf), B, T, H, W, D, ptr(weight), ptr(bias), mode, ptr(outf),
         ptr(outb), ptr(part), stream_ptr())
    mean = torch.empty(M, device=xb.device, dtype=F32)
    rstd = torch.empty(M, device=xb.device, dtype=F32)
    call('ctclip_ln_stats_merge', ptr(part), D // 64, M, D, float(eps), ptr(mean), ptr(rstd), stream_ptr())
    return outf, outb, mean, rstd


def skinny_linear(x, w):
    """y[M, N] f32 = x[M, K] @ w[N, K]^T for M <= 16 rows, both bf16 (ctclip_skinny_gemm) or both f32
    (ctclip_skinny_sgemm, an f32 fma per product) K-contiguous, through the HBM-streaming skinny GEMM
    (w read once, partial sums per k-slice reduced in a fixed order).  Returns None when the shape
    does not qualify."""
    M, Kd = x.shape
    N = w.shape[0]
    if x.dtype != w.dtype or x.dtype not in (BF16, F32) or x.stride(1) != 1 or w.stride(1) != 1 or w.shape[1] != Kd:
        return None
    name = 'ctclip_skinny_gemm' if x.dtype == BF16 else 'ctclip_skinny_sgemm'
    ns = getattr(_lib.lib(), name + '_slices')(M, N, Kd)
    if ns <= 0:
        return None
    slabs = torch.empty(ns, M, N, device=x.device, dtype=F32)
    call(name, ptr(x), x.stride(0), ptr(w), w.stride(0), M, N, Kd, ptr(slabs), ns, stream_ptr())
    out = torch.empty(M, N, device=x.device, dtype=F32)
    reduce_slabs(slabs, out)
    return out


def peg_fwd_x32(xf, B, T, H, W, weight, bias, mode, stats=False, want_f16=False, eps=1e-5, want_x3=False,
                want_bf16=True):
    """PEG forward with the taps read from the f32 residual stream (ctclip_peg_fwd_x32; the bf16
    shadow's rounding never enters the conv).  Returns (out_f32, out_bf16, out_f16 or None, mean,
    rstd) -- mean / rstd the LayerNorm statistics of the output rows when stats (merged from the
    kernel's 32-channel groups), else None; with want_x3 the third entry is the output's split-fp16
    pair (hi, lo) (the x3 Q | K | V GEMM's A operand).  The fp16 outputs are range-checked into the
    step status word (CT_STATUS_F16_RANGE)."""
    M, D = xf.shape
    assert xf.dtype == F32 and xf.is_contiguous()
    outf = torch.empty_like(xf)
    outb = torch.empty(M, D, device=xf.device, dtype=BF16) if want_bf16 else None
    outh = torch.empty(M, D, device=xf.device, dtype=torch.float16) if want_f16 or want_x3 else None
    outl = torch.empty(M, D, device=xf.device, dtype=torch.float16) if want_x3 else None
    part = torch.empty(D // 32, M, 2, device=xf.device, dtype=F32) if stats else None
    call('ctclip_peg_fwd_x32s', ptr(xf), B, T, H, W, D, ptr(weight), ptr(bias), mode, ptr(outf), ptr(outb), ptr(outh),
         ptr(outl), ptr(part), ptr(status_word(xf.device)) if outh is not None else None, stream_ptr())
    if want_x3:
        outh = (outh, outl)
    if not stats:
        return outf, outb, outh, None, None
    mean = torch.empty(M, device=xf.device, dtype=F32)
    rstd = torch.empty(M, device=xf.device, dtype=F32)
    call('ctclip_ln_stats_merge', ptr(part), D // 32, M, D, float(eps), ptr(mean), ptr(rstd), stream_ptr())
    return outf, outb, outh, mean, rstd


def pack_qkv_fold(wq, gamma, wkv_b, s_fold, s_rest):
    """[bf16(Wq o gamma) ; Wkv], the f32 row sums of the folded rows and the concatenated
    l2norm scales [s_fold ; s_rest] (ctclip_pack_qkv_fold, one launch)."""
    nq, K = wq.shape
    nr = wkv_b.shape[0]
    assert wq.dtype == F32 and wq.stride(1) == 1 and gamma.numel() == K and wkv_b.dtype == BF16
    assert s_fold.numel() == s_rest.numel() and s_fold.is_contiguous() and s_rest.is_contiguous()
    out = torch.empty(nq + nr, K, device=wq.device, dtype=BF16)
    cs = torch.empty(nq, device=wq.device, dtype=F32)
    ns = s_fold.numel()
    scales = torch.empty(2 * ns, device=wq.device, dtype=F32)
    g = gamma.detach().contiguous()
    call('ctclip_pack_qkv_fold', ptr(wq), wq.stride(0), ptr(g), nq, K, ptr(wkv_b), wkv_b.stride(0), nr, ptr(out),
         out.stride(0), ptr(cs), ptr(s_fold), ptr(s_rest), ns, ptr(scales), stream_ptr())
    return out, cs, scales


def pack_qkv_fold_h16(wq, gamma, wkv):
    """fp16 [f16(Wq o gamma) ; f16(Wkv)] and the f32 row sums of its folded rows (the fp16 GEMM's fold
    constants; ctclip_pack_qkv_fold_h16).  wq, wkv f32."""
    nq, K = wq.shape
    nr = wkv.shape[0]
    assert wq.dtype == F32 and wkv.dtype == F32 and wq.stride(1) == 1 and wkv.stride(1) == 1
    out = torch.empty(nq + nr, K, device=wq.device, dtype=F16)
    cs = torch.empty(nq, device=wq.device, dtype=F32)
    g = gamma.detach().contiguous()
    call('ctclip_pack_qkv_fold_h16', ptr(wq), wq.stride(0), ptr(g), nq, K, ptr(wkv), wkv.stride(0), nr, ptr(out),
         out.stride(0), ptr(cs), stream_ptr())
    return out, cs


def linear_qkv_lnfold(x, wp, cs, mean, rstd, scales, nfold, n2, out=None, out2=None, c_col0=0):
    """C = x @ wp^T with the LayerNorm folded into columns < nfold and the per-head l2norm * scale
    of columns < n2 in C2 (ctclip_gemm_qkv_lnfold); scales = [64] f32 (folded columns' 32, then
    the rest's).  Returns (C [M, N] bf16, C2 [M, n2] bf16); c_col0 > 0: C's columns below it are not
    written (the eval forward keeps only V, ctclip_gemm_qkv_lnfold2)."""
    M, K = x.shape
    N = wp.shape[0]
    assert wp.shape[1] == K and x.stride(1) == 1 and wp.stride(1) == 1 and scales.numel() == 64
    if out is None:
        out = torch.empty(M, N, device=x.device, dtype=BF16)
    if out2 is None:
        out2 = torch.empty(M, n2, device=x.device, dtype=BF16)
    a = GemmArgs()
    a.M, a.N, a.K = M, N, K
    a.A, a.lda, a.a_kcontig = ptr(x), x.stride(0), 1
    a.B, a.ldb, a.b_kcontig = ptr(wp), wp.stride(0), 1
    a.C, a.ldc, a.c_f32 = ptr(out), out.stride(0), 0
    a.C2, a.ldc2 = ptr(out2), out2.stride(0)
    a.bias = ptr(scales)
    a.alpha, a.act, a.split_k, a.batch = 1.0, ACT_L2N, 1, 1
    a.n2 = n2
    assert wp.dtype == x.dtype
    a.ab_f16 = int(x.dtype == F16)     # fp16 x and packed weight (pack_qkv_fold_h16)
    call('ctclip_gemm_qkv_lnfold2', _lib.ctypes.byref(a), ptr(mean), ptr(rstd), ptr(cs), nfold, int(c_col0),
         stream_ptr())
    return out, out2


def l2norm_scale_bwd_fold(x, dy, H, D, scale, row_rstd, row_mean, *, out=None, dx2=None, fold_cs=None, Dm=0,
                          ds_out=None):
    """l2norm_scale_bwd for the folded-LayerNorm Q (x = the forward's q): dx into `out` (optional),
    dx2 = bf16(dx o rstd) (written into `dx2` when given, e.g. a column slice of the [dq2 | dk | dv]
    buffer), u = dx2^T mean [H D]; with fold_cs / Dm also the LayerNorm backward's row terms (c1,
    beta) of ctclip_gemm_lnfold_bwd.  Returns (dscale or ds_out, dx2, u, c1, beta)."""
    rows = x.shape[0]
    lpr = H * D // 8
    nb = 2048
    while (nb * 256) % lpr:
        nb += 1
    part = torch.empty(nb, D, device=x.device, dtype=F32)
    if dx2 is None:
        dx2 = torch.empty(rows, H * D, device=x.device, dtype=BF16)
    part_u = torch.empty(nb, H * D, device=x.device, dtype=F32)
    c1 = beta = None
    if fold_cs is not None:
        c1 = torch.empty(rows, device=x.device, dtype=F32)
        beta = torch.empty(rows, device=x.device, dtype=F32)
    call('ctclip_l2norm_scale_bwd_fold', ptr(x), x.stride(0), ptr(dy), dy.stride(0), rows, H, D, ptr(scale),
         ptr(out), out.stride(0) if out is not None else 0, ptr(part), nb, ptr(row_rstd), ptr(row_mean), ptr(dx2),
         dx2.stride(0), ptr(part_u), ptr(fold_cs), int(Dm), ptr(c1), ptr(beta), stream_ptr())
    u = torch.empty(H * D, device=x.device, dtype=F32)
    reduce_slabs(part_u.view(nb, 1, H * D), u.view(1, H * D))
    if ds_out is not None:
        ds = reduce_param_partials(part, ds_out, True)
    else:
        ds = torch.empty(D, device=x.device, dtype=F32)
        reduce_slabs(part.view(nb, 1, D), ds.view(1, D))
    return ds, dx2, u, c1, beta


def l2norm_qk_bwd_fold(qk, dqk, q_scale, k_scale, row_rstd, row_mean, out, fold_cs, Dm, ds_q_out=None,
                       ds_k_out=None):
    """Both l2norm backwards of the folded layer (ctclip_l2norm_qk_bwd_fold): qk = the forward's
    [q | k] (256 + 256 columns), dqk = [dq_n | dk_n]; writes [dq o rstd | dk] into `out`.  Returns
    (ds_q, ds_k, u, c1, beta); ds_* accumulate into the given sinks (deferred in a backward)."""
    rows = qk.shape[0]
    assert qk.shape[1] == 512 and dqk.shape[1] == 512 and out.shape[1] == 512
    nb = 1024    # the u partials are summed right away (lnfold_wgrad reads u): fewer, longer blocks
    dev = qk.device
    part_s = torch.empty(2, nb, 32, device=dev, dtype=F32)
    part_u = torch.empty(nb, 256, device=dev, dtype=F32)
    c1 = torch.empty(rows, device=dev, dtype=F32)
    beta = torch.empty(rows, device=dev, dtype=F32)
    call('ctclip_l2norm_qk_bwd_fold', ptr(qk), qk.stride(0), ptr(dqk), dqk.stride(0), rows, ptr(q_scale),
         ptr(k_scale), ptr(out), out.stride(0), ptr(part_s), nb, ptr(row_rstd), ptr(row_mean), ptr(part_u),
         ptr(fold_cs), int(Dm), ptr(c1), ptr(beta), stream_ptr())
    u = torch.empty(256, device=dev, dtype=F32)
    reduce_slabs(part_u.view(nb, 1, 256), u.view(1, 256))
    ds = []
    for i, sink in ((0, ds_q_out), (1, ds_k_out)):
        if sink is not None:
            ds.append(reduce_param_partials(part_s[i], sink, True))
        else:
            d = torch.empty(32, device=dev, dtype=F32)
            reduce_slabs(part_s[i].view(nb, 1, 32), d.view(1, 32))
            ds.append(d)
    return ds[0], ds[1], u, c1, beta


def lnfold_wgrad(G, u, gamma, grad_q, *, wq=None, grad_gamma=None, grad_rest=None):
    """Weight gradients of the fold from G = [dq o rstd | dkv]^T x ([nq + nrest, K] f32):
    grad_q += gamma o (G[:nq] - u), grad_gamma += sum_n wq o (G[:nq] - u) (optional),
    grad_rest += G[nq:] (ctclip_lnfold_wgrad)."""
    nq = grad_q.shape[0]
    Kd = G.shape[1]
    nrest = G.shape[0] - nq
    assert nrest == 0 or grad_rest is not None
    g = gamma.detach().contiguous()
    call('ctclip_lnfold_wgrad', ptr(G), G.stride(0), ptr(u), ptr(g), ptr(wq), wq.stride(0) if wq is not None else 0,
         nq, nrest, Kd, ptr(grad_q), grad_q.stride(0), ptr(grad_gamma), ptr(grad_rest),
         grad_rest.stride(0) if grad_rest is not None else 0, stream_ptr())
    return grad_q


def matmul_lnfold_bwd(dqkv, wp, res, x, c1, beta, out=None, out2=None):
    """dx = [dq o rstd | dk | dv] @ [gamma o Wq ; Wkv] + res - c1 - beta o x (f32) and its bf16 copy:
    the folded LayerNorm's backward through the Q | K | V projections (ctclip_gemm_lnfold_bwd)."""
    M, Kq = dqkv.shape
    N = wp.shape[1]
    assert wp.shape[0] == Kq and dqkv.stride(1) == 1 and wp.stride(1) == 1
    if out is None:
        out = torch.empty(M, N, device=dqkv.device, dtype=F32)
    if out2 is None:
        out2 = torch.empty(M, N, device=dqkv.device, dtype=BF16)
    a = GemmArgs()
    a.M, a.N, a.K = M, N, Kq
    a.A, a.lda, a.a_kcontig = ptr(dqkv), dqkv.stride(0), 1
    a.B, a.ldb, a.b_kcontig = ptr(wp), wp.stride(0), 0
    a.C, a.ldc, a.c_f32 = ptr(out), out.stride(0), 1
    a.C2, a.ldc2 = ptr(out2), out2.stride(0)
    a.R, a.ldr, a.r_f32 = ptr(res), res.stride(0), 1
    a.alpha, a.act, a.split_k, a.batch = 1.0, ACT_NONE, 1, 1
    call('ctclip_gemm_lnfold_bwd', _lib.ctypes.byref(a), ptr(x), x.stride(0), ptr(c1), ptr(beta), stream_ptr())
    return out, out2


def peg_bwd(doutb, doutf, xb, B, T, H, W, weight, mode, dweight_out=None, dbias_out=None):
    """Returns (dx_f32, dx_bf16, dweight [D,27], dbias [D]).  dweight_out / dbias_out (the
    parameters' .grad, [D, 27]-contiguous / [D]): the weight gradient accumulates into them in the
    same launch that sums the partial slabs (ctclip_peg_wgrad_reduce) and the returned dweight /
    dbias are those sinks."""
    D = xb.shape[1]
    dxf = torch.empty_like(doutf)
    dxb = torch.empty_like(doutb)
    # the input gradient from the f32 dout alone (conv taps in f32) where the x32 kernel takes the
    # shape; else the bf16-tap tile kernel (CTCLIP_PEG_BWD_X32=0: always the latter, A/B)
    rc = _CT_ESHAPE
    if _PEG_BWD_X32 and doutf.is_contiguous():
        rc = _lib.lib().ctclip_peg_bwd_data_x32(ptr(doutf), B, T, H, W, D, ptr(weight), mode, ptr(dxf), ptr(dxb),
                                                stream_ptr())
    if rc == _CT_ESHAPE:
        call('ctclip_peg_bwd_data', ptr(doutb), ptr(doutf), B, T, H, W, D, ptr(weight), mode, ptr(dxf), ptr(dxb),
             stream_ptr())
    elif rc != 0:
        raise _lib.KernelError(f'ctclip_peg_bwd_data_x32 failed with code {rc}')
    nblk = _lib.lib().ctclip_peg_wgrad_slabs(B, T, H, W, D)
    part = torch.empty(nblk, D * 28, device=xb.device, dtype=F32)
    call('ctclip_peg_bwd_weight', ptr(doutb), ptr(xb), B, T, H, W, D, mode, ptr(part), nblk, stream_ptr())
    if dweight_out is not None or dbias_out is not None:
        assert dweight_out is None or (dweight_out.is_contiguous() and dweight_out.numel() == D * 27)
        assert dbias_out is None or (dbias_out.is_contiguous() and dbias_out.numel() == D)
        call('ctclip_peg_wgrad_reduce', ptr(part), nblk, D, ptr(dweight_out), ptr(dbias_out), 1, stream_ptr())
        return dxf, dxb, dweight_out, dbias_out
    dw = torch.empty(D, 27, device=xb.device, dtype=F32)
    db = torch.empty(D, device=xb.device, dtype=F32)
    call('ctclip_peg_wgrad_reduce', ptr(part), nblk, D, ptr(dw), ptr(db), 0, stream_ptr())
    return dxf, dxb, dw, db


# ----------------------------------------------------------------------------- attention
def _attn_args(q, k, v, o, *, L, H, D, nseq, M, scale, seq, bias_u=None, grid=(0, 0), kmask=None, lse=None,
               dout=None, dq=None, dk=None, dv=None, delta=None, dbias_u=None, dropout=(0.0, 0)):
    a = _lib.AttnArgs()
    a.q, a.ldq = ptr(q), q.stride(0)
    a.k, a.ldk = ptr(k), k.stride(0)
    a.v, a.ldv = ptr(v), v.stride(0)
    a.o, a.ldo = ptr(o), o.stride(0)
    a.dout, a.lddo = ptr(dout), dout.stride(0) if dout is not None else 0
    a.dq, a.lddq = ptr(dq), dq.stride(0) if dq is not None else 0
    a.dk, a.lddk = ptr(dk), dk.stride(0) if dk is not None else 0
    a.dv, a.lddv = ptr(dv), dv.stride(0) if dv is not None else 0
    a.lse, a.delta = ptr(lse), ptr(delta)
    a.bias_u, a.dbias_u, a.kmask = ptr(bias_u), ptr(dbias_u), ptr(kmask)
    a.scale, a.L, a.H, a.D, a.nseq, a.M = scale, L, H, D, nseq, M
    a.grid_h, a.grid_w = grid
    a.n_inner, a.s_outer, a.s_inner, a.s_pos = seq
    a.dropout_p, a.dropout_seed = float(dropout[0]), int(dropout[1]) & (2 ** 64 - 1)
    return a


def attn_fwd(q, k, v, *, L, H, D, nseq, scale, seq, bias_u=None, grid=(0, 0), kmask=None, dropout=(0.0, 0),
             want_o16=False, eval_only=False):
    """q/k/v: 2D views [M, ...] whose head h occupies columns h*D:(h+1)*D.  Returns (o [M, H*D], lse [H, M]),
    plus o's fp16 copy when want_o16.  eval_only (with want_o16): neither the bf16 o nor the lse -- the
    backward's operands -- is written (returned as None)."""
    M = q.shape[0]
    assert want_o16 or not eval_only
    o = None if eval_only else torch.empty(M, H * D, device=q.device, dtype=BF16)
    o16 = torch.empty(M, H * D, device=q.device, dtype=F16) if want_o16 else None
    lse = None if eval_only else torch.empty(H, M, device=q.device, dtype=F32)
    a = _attn_args(q, k, v, o if o is not None else o16, L=L, H=H, D=D, nseq=nseq, M=M, scale=scale, seq=seq,
                   bias_u=bias_u, grid=grid, kmask=kmask, lse=lse, dropout=dropout)
    if o is None:
        a.o = None
    a.o16 = ptr(o16)
    call('ctclip_attn_fwd', _lib.ctypes.byref(a), stream_ptr())
    return (o, lse, o16) if want_o16 else (o, lse)


def attn_bwd(q, k, v, o, lse, dout, dq, dk, dv, *, L, H, D, nseq, scale, seq, bias_u=None, dbias_u=None,
             grid=(0, 0), kmask=None, dropout=(0.0, 0)):
    M = q.shape[0]
    delta = torch.empty(H, M, device=q.device, dtype=F32)
    a = _attn_args(q, k, v, o, L=L, H=H, D=D, nseq=nseq, M=M, scale=scale, seq=seq, bias_u=bias_u, grid=grid,
                   kmask=kmask, lse=lse, dout=dout, dq=dq, dk=dk, dv=dv, delta=delta, dbias_u=dbias_u,
                   dropout=dropout)
    ws = None
    if dbias_u is not None and _ATTN_BIAS_WS:
        # per-workgroup partial bins + one deterministic reduction instead of global float atomics
        n = _lib.lib().ctclip_attn_bwd_ws_floats(_lib.ctypes.byref(a))
        if n > 0:
            ws = torch.empty(n, device=q.device, dtype=F32)
            a.dbias_ws, a.dbias_ws_floats = ptr(ws), n
    call('ctclip_attn_bwd', _lib.ctypes.byref(a), stream_ptr())


# the bias-gradient workspace (deterministic slab reduction) costs within noise of the global
# float atomics (spatial backward 822 vs 810 us, profiles/r02bc_attn_ws_ab.log) and makes the bias
# gradient bit-reproducible: default since round 3 (CTCLIP_ATTN_BIAS_WS=0 = the atomics)
_ATTN_BIAS_WS = os.environ.get('CTCLIP_ATTN_BIAS_WS', '1') != '0'


# ----------------------------------------------------------------------------- VQ
def vq_select(cand, x, codebook_f32, margin=2e-2, want_xn=True, cand2=None):
    """Exact f32 cosine argmax from the bf16 GEMM's per-group candidates (vq.hip); cand2 = the
    groups' second-best scores (None: group winners only)."""
    rows, D = x.shape
    idx = torch.empty(rows, device=x.device, dtype=torch.int32)
    xn = torch.empty(rows, D, device=x.device, dtype=F32) if want_xn else None
    # a token without a finite score sets CT_STATUS_VQ_NONFINITE in the step status word
    call('ctclip_vq_select_s', ptr(cand), ptr(cand2), cand.shape[1], ptr(x), rows, D, ptr(codebook_f32),
         codebook_f32.shape[0], margin, ptr(idx), ptr(xn), ptr(status_word(x.device)), stream_ptr())
    return idx, xn


def vq_l2norm_h16(x):
    """fp16 l2norm of the f32 tokens [rows, D] (ctclip_vq_l2norm_h16): the fp16 VQ distance GEMM's A."""
    rows, D = x.shape
    assert x.dtype == F32 and x.stride(1) == 1
    y = torch.empty(rows, D, device=x.device, dtype=F16)
    call('ctclip_vq_l2norm_h16', ptr(x), x.stride(0), rows, D, ptr(y), D, stream_ptr())
    return y


def vq_pool(idx, codebook_f32, B, T, HW, want_bf16=True):
    D = codebook_f32.shape[1]
    out = torch.empty(B, HW * D, device=idx.device, dtype=F32)
    outb = torch.empty(B, HW * D, device=idx.device, dtype=BF16) if want_bf16 else None
    call('ctclip_vq_pool', ptr(idx), ptr(codebook_f32), B, T, HW, D, ptr(out), ptr(outb), stream_ptr())
    return out, outb


def vq_pool_bwd(dpooled, B, T, HW, D):
    dx = torch.empty(B * T * HW, D, device=dpooled.device, dtype=F32)
    dxb = torch.empty(B * T * HW, D, device=dpooled.device, dtype=BF16)
    call('ctclip_vq_pool_bwd', ptr(dpooled), B, T, HW, D, ptr(dx), ptr(dxb), stream_ptr())
    return dx, dxb


def vq_gather(idx, codebook_f32):
    D = codebook_f32.shape[1]
    out = torch.empty(idx.numel(), D, device=idx.device, dtype=F32)
    call('ctclip_vq_gather', ptr(idx), ptr(codebook_f32), idx.numel(), D, ptr(out), stream_ptr())
    return out


def vq_ema_accum(idx, xn, bins, esum, work=None):
    """bins (f32 counts) and esum (int64 [C][D], token sums in 2^-40 fixed point: bit-identical
    whatever order the adds land in) accumulate the EMA statistics of rows xn (unit vectors).
    work: int32 scratch of at least 2 C + 2 rows entries whose first C are zero (left zero): the
    code-sorted kernels (ctclip_vq_ema_accum_sorted, ~10x fewer atomics); None: token order."""
    assert esum.dtype == torch.int64 and bins.dtype == F32
    # the 2^-40 fixed-point sums stay exact while every code's GLOBAL row count (summed over ranks
    # by dist_sync.sum_codebook_stats) is below 2^23; the f32 bins are exact below 2^24
    from . import dist_sync
    if xn.shape[0] * dist_sync.world_rank()[0] >= (1 << 23):
        raise ValueError(f'vq_ema_accum: {xn.shape[0]} rows x {dist_sync.world_rank()[0]} ranks may exceed the 2^23 '
                         'rows per code that the int64 2^-40 fixed-point sums hold exactly')
    if work is not None:
        C = esum.shape[0]
        assert work.dtype == torch.int32 and work.numel() >= 2 * C + 2 * xn.shape[0]
        call('ctclip_vq_ema_accum_sorted', ptr(idx), ptr(xn), xn.shape[0], xn.shape[1], C, ptr(bins), ptr(esum),
             ptr(work), stream_ptr())
        return
    call('ctclip_vq_ema_accum', ptr(idx), ptr(xn), xn.shape[0], xn.shape[1], ptr(bins), ptr(esum), stream_ptr())


def vq_ema_finalize(bins, esum, decay, embed, cluster, embed_bf16=None, reset=False, guard=None):
    """reset: zero bins / esum behind the reads (persistent statistics buffers).  guard (f32 [1], with
    reset): a nonzero value drops this update (embed / cluster untouched, statistics zeroed)."""
    assert esum.dtype == torch.int64
    C, D = esum.shape
    if guard is not None:
        assert reset and guard.dtype == F32
        call('ctclip_vq_ema_finalize_guard', ptr(bins), ptr(esum), C, D, decay, ptr(embed), ptr(cluster),
             ptr(embed_bf16), ptr(guard), stream_ptr())
        return
    call('ctclip_vq_ema_finalize_reset' if reset else 'ctclip_vq_ema_finalize', ptr(bins), ptr(esum), C, D, decay,
         ptr(embed), ptr(cluster), ptr(embed_bf16), stream_ptr())


# ----------------------------------------------------------------------------- loss
def clip_loss(t_raw, i_raw, log_temp):
    Bg, Dl = t_raw.shape
    dev = t_raw.device
    tn = torch.empty_like(t_raw)
    inn = torch.empty_like(i_raw)
    loss = torch.empty(1, device=dev, dtype=F32)
    dt = torch.empty_like(t_raw)
    di = torch.empty_like(i_raw)
    dlt = torch.empty(1, device=dev, dtype=F32)
    sim = torch.empty(Bg, Bg, device=dev, dtype=F32)
    call('ctclip_clip_loss', ptr(t_raw), ptr(i_raw), Bg, Dl, ptr(log_temp), ptr(tn), ptr(inn), ptr(loss), ptr(dt),
         ptr(di), ptr(dlt), ptr(sim), stream_ptr())
    return loss, dt, di, dlt, tn, inn, sim


def zero_shot(t_raw, i_raw, log_temp):
    """Raw prompt latents [2P, Dl] (pairs present / not present) x raw image latents [N, Dl] ->
    (probs [N, P], scores [N, P, 2]); ct_clip/ctclip_inference.py:305-315."""
    P2, Dl = t_raw.shape
    N = i_raw.shape[0]
    if P2 % 2 or i_raw.shape[1] != Dl:
        raise ValueError(f'zero_shot: prompt latents {tuple(t_raw.shape)} must be pairs of {tuple(i_raw.shape)} rows')
    t_raw, i_raw = t_raw.float().contiguous(), i_raw.float().contiguous()
    scores = torch.empty(N, P2 // 2, 2, device=t_raw.device, dtype=F32)
    probs = torch.empty(N, P2 // 2, device=t_raw.device, dtype=F32)
    call('ctclip_zero_shot', ptr(t_raw), ptr(i_raw), P2 // 2, N, Dl, ptr(log_temp.float().contiguous()), ptr(scores),
         ptr(probs), stream_ptr())
    return probs, scores


def clip_scores(t_raw, i_raw, log_temp):
    B, Dl = t_raw.shape
    if i_raw.shape[0] != B:
        # einsum('b d, b d -> b') broadcasts a batch-1 operand (the zero-shot call,
        # ct_clip/ctclip_inference.py:310: 2 prompts x 1 volume)
        if i_raw.shape[0] != 1:
            raise ValueError(f'clip_scores: batch {B} vs {i_raw.shape[0]} do not broadcast')
        i_raw = i_raw.expand(B, Dl).contiguous()
    out = torch.empty(B, device=t_raw.device, dtype=F32)
    call('ctclip_clip_scores', ptr(t_raw), ptr(i_raw), B, Dl, ptr(log_temp), ptr(out), stream_ptr())
    return out


# ----------------------------------------------------------------------------- sgemm
def sgemm(M, N, K, A, sam, sak, B, sbk, sbn, C, scm, scn, *, bias=None, alpha=1.0, act=0, slope=0.1, aux=None,
          sxm=0, sxn=0, accumulate=False):
    # split K when the output has few 64x64 tiles and K is long (CPB weight gradients, K = 2,209)
    tiles = ((M + 63) // 64) * ((N + 63) // 64)
    split = 1
    if K >= 512 and tiles < 128:
        split = max(1, min(K // 128, 256 // tiles))
    ws = torch.empty(split * M * N, device=A.device, dtype=F32) if split > 1 else None
    call('ctclip_sgemm', M, N, K, ptr(A), sam, sak, ptr(B), sbk, sbn, ptr(C), scm, scn, ptr(bias), alpha, act, slope,
         ptr(aux), sxm, sxn, int(accumulate), ptr(ws), split, stream_ptr())
    return C


def slinear(x, w, bias=None, act=0, slope=0.1, out=None, accumulate=False):
    """f32 y = x @ w^T (+b), x [M,K], w [N,K] (any strides)."""
    M, K = x.shape
    N = w.shape[0]
    if out is None:
        out = torch.empty(M, N, device=x.device, dtype=F32)
    return sgemm(M, N, K, x, x.stride(0), x.stride(1), w, w.stride(1), w.stride(0), out, out.stride(0),
                 out.stride(1), bias=bias, act=act, slope=slope, accumulate=accumulate)


def smm(a, b, out=None, accumulate=False, act=0, slope=0.1, aux=None):
    """f32 out = a @ b for 2D strided views; act=2 multiplies by LeakyReLU'(aux)."""
    M, K = a.shape
    N = b.shape[1]
    if out is None:
        out = torch.empty(M, N, device=a.device, dtype=F32)
    return sgemm(M, N, K, a, a.stride(0), a.stride(1), b, b.stride(0), b.stride(1), out, out.stride(0),
                 out.stride(1), act=act, slope=slope, aux=aux, sxm=aux.stride(0) if aux is not None else 0,
                 sxn=aux.stride(1) if aux is not None else 0, accumulate=accumulate)


# ----------------------------------------------------------------------------- BERT embeddings
def embed_fwd(ids, word, pos, type0):
    B, L = ids.shape
    Hd = word.shape[1]
    out = torch.empty(B * L, Hd, device=ids.device, dtype=F32)
    call('ctclip_embed_fwd', ptr(ids), B, L, Hd, ptr(word), ptr(pos), ptr(type0), ptr(out), stream_ptr())
    return out


def embed_bwd(ids, dx, dword, dpos, dtype0, pad_id=-1):
    """Accumulate the embedding-table gradients (no float atomics: bit-reproducible); the rows of
    tokens with id == pad_id add nothing to dword (nn.Embedding padding_idx)."""
    B, L = ids.shape
    call('ctclip_embed_bwd', ptr(ids), B, L, dx.shape[1], ptr(dx), ptr(dword), ptr(dpos), ptr(dtype0), pad_id,
         stream_ptr())


# ----------------------------------------------------------------------------- optimizer
def grad_norm(g, max_norm, out, skip=None):
    """out[0] = ||g||, out[1] = the clip coefficient; skip (device int32[1]): a non-finite norm ORs
    CT_STATUS_NONFINITE_GRAD (4) into it (the Adam kernels' guard word)."""
    nblk = 1024
    part = torch.empty(nblk, device=g.device, dtype=F32)
    call('ctclip_grad_norm_s', ptr(g), g.numel(), max_norm, ptr(part), nblk, ptr(out), ptr(skip), stream_ptr())
    return out


_WEIGHTS_EPOCH = [0]


def weights_epoch():
    """Bumped by every optimizer update: the Adam kernel writes parameters through raw pointers,
    invisible to torch's version counters, so caches of derived weights (bf16 copies) key on
    (data_ptr, _version, weights_epoch())."""
    return _WEIGHTS_EPOCH[0]


def adam(p, g, m, v, *, lr, b1, b2, eps, wd, step, coef=None, p_bf16=None, p_bf16_lo=None, zero_grad=False,
         skip=None):
    """skip: optional device int32[1] guard word; when nonzero the launch changes nothing."""
    assert skip is None or (skip.dtype == torch.int32 and skip.is_cuda)
    call('ctclip_adam', ptr(p), ptr(g), ptr(m), ptr(v), p.numel(), lr, b1, b2, eps, wd, step, ptr(coef), ptr(p_bf16),
         ptr(p_bf16_lo), int(zero_grad), ptr(skip), stream_ptr())
    _WEIGHTS_EPOCH[0] += 1


def gelu_f32(x):
    y = torch.empty_like(x)
    call('ctclip_gelu_f32', ptr(x), ptr(y), x.numel(), stream_ptr())
    return y


def colsum_rows_mean(x, B):
    """x [B*n, D] f32 -> (B, D) mean over each batch's n rows (f32 GEMM against a ones row)."""
    rows, D = x.shape
    n = rows // B
    out = torch.empty(B, D, device=x.device, dtype=F32)
    ones = torch.ones(n, device=x.device, dtype=F32)
    for b in range(B):
        xb = x[b * n:(b + 1) * n]
        sgemm(1, D, n, ones, 0, 1, xb, xb.stride(0), 1, out[b:b + 1], D, 1, alpha=1.0 / n)
    return out


# ---------------------------------------------------------------- MX-fp8 (configs[3])
def quant_mxfp8(x, Kp=None):
    """x [rows, K] bf16 / f32 -> (q [rows, Kp] uint8 e4m3, scales [rows, Kp/32] uint8 e8m0), the
    OCP MX rule of csrc/mxfp8.hip; Kp = K rounded up to 128 (zero-filled)."""
    assert x.dim() == 2 and x.stride(1) == 1 and x.dtype in (torch.bfloat16, torch.float32)
    rows, Kx = x.shape
    Kp = Kp or (Kx + 127) // 128 * 128
    q = torch.empty(rows, Kp, device=x.device, dtype=torch.uint8)
    s = torch.empty(rows, Kp // 32, device=x.device, dtype=torch.uint8)
    call('ctclip_quant_mxfp8', ptr(x), int(x.dtype == torch.float32), rows, Kx, x.stride(0), ptr(q), q.stride(0),
         ptr(s), Kp, stream_ptr())
    return q, s


def gemm_mxfp8(qa, sa, qb, sb, *, bias=None, alpha=1.0, out_f32=False, out=None, residual=None, out2=None,
               act=ACT_NONE):
    """C[M, N] = alpha * dequant(qa) . dequant(qb)^T (+ bias) (+ f32 residual) from quant_mxfp8
    operands; out2: bf16 copy of C, or with act=ACT_GEGLU the GEGLU output g [M, N/2] (C = h)."""
    M, Kp = qa.shape
    N = qb.shape[0]
    assert qb.shape[1] == Kp and sa.shape == (M, Kp // 32) and sb.shape == (N, Kp // 32)
    assert act in (ACT_NONE, ACT_GEGLU)
    C = out if out is not None else torch.empty(M, N, device=qa.device,
                                                dtype=torch.float32 if out_f32 else torch.bfloat16)
    if residual is not None:
        assert residual.dtype == torch.float32 and residual.shape == (M, N) and residual.stride(1) == 1
    a = _lib.MxGemmArgs(M=M, N=N, Kp=Kp, A=ptr(qa), lda=qa.stride(0), sA=ptr(sa), B=ptr(qb), ldb=qb.stride(0),
                        sB=ptr(sb), C=ptr(C), ldc=C.stride(0), c_f32=int(C.dtype == torch.float32),
                        bias=ptr(bias), alpha=float(alpha), R=ptr(residual),
                        ldr=residual.stride(0) if residual is not None else 0, C2=ptr(out2),
                        ldc2=out2.stride(0) if out2 is not None else 0, act=int(act))
    call('ctclip_gemm_mxfp8', _lib.ctypes.byref(a), stream_ptr())
    return C


def gemm_mxfp8_set_tile(bm):
    """diagnostic: force the 128- / 256-row MX tile kernel (0 = auto); returns the previous."""
    return _lib.lib().ctclip_gemm_mxfp8_set_tile(int(bm))


def dropout(x, p, seed, *, res=None, out_f32=True, out_bf16=False):
    """BERT hidden dropout: (x * keep / (1 - p) (+ res)) as (f32 or None, bf16 or None)."""
    assert x.dtype == F32 and x.is_contiguous() and (res is None or (res.dtype == F32 and res.is_contiguous()))
    yf = torch.empty_like(x) if out_f32 else None
    yb = torch.empty(x.shape, device=x.device, dtype=BF16) if out_bf16 else None
    call('ctclip_dropout', ptr(x), ptr(res), ptr(yf), ptr(yb), x.numel(), float(p), int(seed) & (2 ** 64 - 1),
         stream_ptr())
    return yf, yb


# ---------------------------------------------------------------- f32 image tower (precise.py)
def patch_ln_f32(video, is_hu, PT, P, offs, gamma, beta, eps=1e-5):
    """to_patch_emb's Rearrange + LayerNorm(pd) with affine, f32 rows [tokens, pd]."""
    B, C, Fr, H, W = video.shape
    T, Hg, Wg = Fr // PT, H // P, W // P
    pd = C * PT * P * P
    out = torch.empty(B * T * Hg * Wg, pd, device=video.device, dtype=F32)
    call('ctclip_patch_ln_f32', ptr(video), int(video.dtype == F32), int(is_hu), B, C, Fr, H, W, PT, P, ptr(offs),
         eps, ptr(gamma), ptr(beta), ptr(out), pd, stream_ptr())
    return out


def peg_fwd_f32(x, B, T, H, W, weight, bias, mode):
    out = torch.empty_like(x)
    call('ctclip_peg_fwd_f32', ptr(x), B, T, H, W, x.shape[1], ptr(weight), ptr(bias), mode, ptr(out), stream_ptr())
    return out


def l2norm_scale_fwd_f32(x, H, D, scale, out_bf16=None):
    """f32 l2norm * scale per head; out_bf16: also write its bf16 copy there ([rows, H D] view)."""
    out = torch.empty(x.shape[0], H * D, device=x.device, dtype=F32)
    call('ctclip_l2norm_scale_fwd_f32b', ptr(x), x.stride(0), x.shape[0], H, D, ptr(scale), ptr(out), out.stride(0),
         ptr(out_bf16), out_bf16.stride(0) if out_bf16 is not None else 0, stream_ptr())
    return out


def linear_f32(x, w, *, bias=None, residual=None, want_bf16=False, alpha=1.0, out_bf16=None):
    """Exact-f32 y[M, N] = alpha x[M, K] @ w[N, K]^T (+ bias) (+ residual f32) on the f32 MFMA GEMM
    (ctclip_sgemm_tn; one ascending-k fma chain per output).  Returns (y f32, bf16 copy or None);
    out_bf16: the bf16 copy goes into this [M, N] view."""
    M, Kd = x.shape
    N = w.shape[0]
    assert w.shape[1] == Kd and x.dtype == F32 and w.dtype == F32 and x.stride(1) == 1 and w.stride(1) == 1
    y = torch.empty(M, N, device=x.device, dtype=F32)
    yb = out_bf16
    if yb is not None:
        assert yb.dtype == BF16 and yb.shape == (M, N) and yb.stride(1) == 1
    elif want_bf16:
        yb = torch.empty(M, N, device=x.device, dtype=BF16)
    a = _lib.SgemmTnArgs(M=M, N=N, K=Kd, A=ptr(x), lda=x.stride(0), B=ptr(w), ldb=w.stride(0), C=ptr(y), ldc=N,
                         C2=ptr(yb), ldc2=yb.stride(0) if yb is not None else N, C3=None, ldc3=0, bias=ptr(bias),
                         R=ptr(residual),
                         ldr=residual.stride(0) if residual is not None else 0, alpha=float(alpha), act=0)
    call('ctclip_sgemm_tn', _lib.ctypes.byref(a), stream_ptr())
    return y, yb


def linear_f32_geglu(x, w1p):
    """FF1 + GEGLU in exact f32 on the packed [32 x | 32 gate] weight (functional.pack_ff1 order, f32):
    returns (h bf16 [M, N], g f32 [M, N/2], g bf16 [M, N/2])."""
    M, Kd = x.shape
    N = w1p.shape[0]
    assert w1p.shape[1] == Kd and N % 64 == 0 and x.dtype == F32 and w1p.dtype == F32
    h = torch.empty(M, N, device=x.device, dtype=BF16)
    g = torch.empty(M, N // 2, device=x.device, dtype=F32)
    gb = torch.empty(M, N // 2, device=x.device, dtype=BF16)
    a = _lib.SgemmTnArgs(M=M, N=N, K=Kd, A=ptr(x), lda=x.stride(0), B=ptr(w1p), ldb=w1p.stride(0), C=ptr(g),
                         ldc=N // 2, C2=ptr(h), ldc2=N, C3=ptr(gb), ldc3=N // 2, bias=None, R=None, ldr=0, alpha=1.0,
                         act=ACT_GEGLU)
    call('ctclip_sgemm_tn', _lib.ctypes.byref(a), stream_ptr())
    return h, g, gb


def geglu_f32(h):
    rows, two = h.shape
    inner = two // 2
    g = torch.empty(rows, inner, device=h.device, dtype=F32)
    call('ctclip_geglu_f32', ptr(h), h.stride(0), rows, inner, ptr(g), g.stride(0), stream_ptr())
    return g


def attn_fwd_f32(q, k, v, *, L, H, D, nseq, scale, seq, bias_u=None, grid=(0, 0)):
    M = q.shape[0]
    o = torch.empty(M, H * D, device=q.device, dtype=F32)
    a = _attn_args(q, k, v, o, L=L, H=H, D=D, nseq=nseq, M=M, scale=scale, seq=seq, bias_u=bias_u, grid=grid)
    call('ctclip_attn_fwd_f32', _lib.ctypes.byref(a), stream_ptr())
    return o


# ---------------------------------------------------------------- split-fp16 x3 image tower (round 6)
# precise.set_vit_precision('split'): every forward Linear of the 3D-ViT on the x3 GEMM (gemm256.hip,
# ctclip_gemm_args.A_lo / B_lo): operands as fp16 (hi, lo) image pairs, three fp16 MFMA products per
# K-step into one f32 accumulator -- ~22-bit operands at 3x the fp16 MFMA work instead of f32 MFMA
# at 1/16 of the rate (tools/vit_precision.py 's:' / 'S:' sites: pre-VQ 1.2e-6, 0 flips).
X3_WSCALE = 256.0   # weights are packed x256 (their ~1e-2 entries keep a normal fp16 lo part); alpha = 1/256


def status_word(device):
    """The device's sticky int32[1] step status word (include/ctclip_hip.h CT_STATUS_*): the
    LayerNorm exchange timeouts, fp16 range / non-finite flags of the producers that take it."""
    return ln_status_tensor(device)


def split_f16(x, scale=1.0, out=None):
    """(hi, lo) fp16 images of f32 x [rows, cols]: hi = fp16(x s), lo = fp16(x s - hi)."""
    rows, cols = x.shape
    assert x.dtype == F32 and x.stride(1) == 1
    hi, lo = out if out is not None else (torch.empty(rows, cols, device=x.device, dtype=F16),
                                          torch.empty(rows, cols, device=x.device, dtype=F16))
    call('ctclip_split_f16', ptr(x), x.stride(0), rows, cols, float(scale), ptr(hi), ptr(lo), hi.stride(0),
         ptr(status_word(x.device)), stream_ptr())
    return hi, lo


def pack_rows_x3(src, rows_dst, cols_dst, rowmap=None, colscale=None, scale=X3_WSCALE):
    """pack_rows of an f32 weight into its split-fp16 pair, scaled by `scale` (see X3_WSCALE)."""
    rows, cols = src.shape
    assert src.dtype == F32 and src.stride(1) == 1
    hi = torch.empty(rows_dst, cols_dst, device=src.device, dtype=F16)
    lo = torch.empty(rows_dst, cols_dst, device=src.device, dtype=F16)
    call('ctclip_pack_rows_x3', ptr(src), src.stride(0), ptr(rowmap), rows_dst, cols, cols_dst, ptr(colscale),
         float(scale), ptr(hi), ptr(lo), hi.stride(0), ptr(status_word(src.device)), stream_ptr())
    return hi, lo


def _x3_args(xs, ws, C, alpha):
    (xh, xl), (wh, wl) = xs, ws
    M, Kd = xh.shape
    N = wh.shape[0]
    assert xh.dtype == F16 and xl.dtype == F16 and wh.dtype == F16 and wl.dtype == F16
    assert xl.shape == xh.shape and xl.stride() == xh.stride() and wl.shape == wh.shape and wl.stride() == wh.stride()
    assert wh.shape[1] == Kd and xh.stride(1) == 1 and wh.stride(1) == 1 and Kd % 64 == 0
    a = GemmArgs()
    a.M, a.N, a.K = M, N, Kd
    a.A, a.lda, a.a_kcontig = ptr(xh), xh.stride(0), 1
    a.B, a.ldb, a.b_kcontig = ptr(wh), wh.stride(0), 1
    a.A_lo, a.B_lo = ptr(xl), ptr(wl)
    a.C, a.ldc = ptr(C), C.stride(0)
    a.alpha, a.split_k, a.batch, a.ab_f16 = float(alpha), 1, 1, 1
    return a


def linear_x3(xs, ws, *, bias=None, residual=None, want_bf16=False, alpha=1.0 / X3_WSCALE, tag=None, flops=None,
              out_bf16=None):
    """y [M, N] f32 = alpha xs . ws^T (+ bias) (+ f32 residual) on the x3 GEMM, xs / ws split-fp16
    pairs ([M, K] activations, [N, K] weights packed by pack_rows_x3); returns (y, bf16 copy or None).
    out_bf16: write the bf16 copy into this [M, N] view (e.g. columns of a wider buffer)."""
    M, N = xs[0].shape[0], ws[0].shape[0]
    y = torch.empty(M, N, device=xs[0].device, dtype=F32)
    yb = out_bf16
    if yb is not None:
        assert yb.dtype == BF16 and yb.shape == (M, N) and yb.stride(1) == 1
    elif want_bf16:
        yb = torch.empty(M, N, device=y.device, dtype=BF16)
    a = _x3_args(xs, ws, y, alpha)
    a.c_f32 = 1
    a.C2, a.ldc2 = ptr(yb), yb.stride(0) if yb is not None else 0
    a.bias = ptr(bias)
    if residual is not None:
        assert residual.dtype == F32 and residual.shape == (M, N) and residual.stride(1) == 1
        a.R, a.ldr, a.r_f32 = ptr(residual), residual.stride(0), 1
    end = TIMER(tag, flops if flops is not None else 2.0 * M * N * xs[0].shape[1]) if tag else None
    call('ctclip_gemm', _lib.ctypes.byref(a), stream_ptr())
    if end is not None:
        end.record()
    return y, yb


def linear_x3_geglu(xs, w1s, *, alpha=1.0 / X3_WSCALE, want_bf16=True, tag=None, flops=None):
    """FF1 + GEGLU on the x3 GEMM over the packed [32 x | 32 gate] weight pair (functional.pack_ff1
    order): returns (h fp16 [M, N], (g hi, g lo) fp16 [M, N/2] -- FF2's A operand --, g bf16 or None)."""
    M, N = xs[0].shape[0], w1s[0].shape[0]
    assert N % 64 == 0
    dev = xs[0].device
    h = torch.empty(M, N, device=dev, dtype=F16)
    gh = torch.empty(M, N // 2, device=dev, dtype=F16)
    gl = torch.empty(M, N // 2, device=dev, dtype=F16)
    gb = torch.empty(M, N // 2, device=dev, dtype=BF16) if want_bf16 else None
    a = _x3_args(xs, w1s, h, alpha)
    a.act = ACT_GEGLU
    a.C2, a.ldc2 = ptr(gh), N // 2
    a.C3, a.ldc3 = ptr(gl), N // 2
    a.C4, a.ldc4 = ptr(gb), N // 2 if gb is not None else 0
    end = TIMER(tag, flops if flops is not None else 2.0 * M * N * xs[0].shape[1]) if tag else None
    call('ctclip_gemm', _lib.ctypes.byref(a), stream_ptr())
    if end is not None:
        end.record()
    return h, (gh, gl), gb


def attn_fwd_x3(q, k, v, *, L, H, D, nseq, scale, seq, bias_u=None, grid=(0, 0), want_bf16=True, want_lse=True):
    """The cosine attention on split-fp16 x3 MFMAs (ctclip_attn_fwd_x3): q, k, v f32 (head h in columns
    h D .. h D + D - 1).  Returns ((o hi, o lo) fp16 [M, H D], o bf16 or None, lse [H, M] or None)."""
    M = q.shape[0]
    dev = q.device
    oh = torch.empty(M, H * D, device=dev, dtype=F16)
    ol = torch.empty(M, H * D, device=dev, dtype=F16)
    ob = torch.empty(M, H * D, device=dev, dtype=BF16) if want_bf16 else None
    lse = torch.empty(H, M, device=dev, dtype=F32) if want_lse else None
    a = _attn_args(q, k, v, oh, L=L, H=H, D=D, nseq=nseq, M=M, scale=scale, seq=seq, bias_u=bias_u, grid=grid)
    a.o = None
    call('ctclip_attn_fwd_x3', _lib.ctypes.byref(a), ptr(oh), ptr(ol), ptr(ob), ptr(lse), stream_ptr())
    return (oh, ol), ob, lse
