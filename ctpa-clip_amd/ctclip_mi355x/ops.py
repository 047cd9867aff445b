"""``torch.library`` custom ops over the C-ABI ("wrapped by torch.library custom ops
with autograd Functions inside ctclip_mi355x").  Namespace ``ctclip``; each op launches the HIP
kernels of ``kernels.py`` on torch's current stream, has a fake (meta) implementation for shape
propagation, and the differentiable ones register their backward with ``register_autograd``.

The model itself runs the fused autograd Functions of ``functional.py`` (one Function per
transformer layer, parameter gradients written straight into the flat gradient arena); these ops
are the same kernels exposed one operation at a time, for callers that compose their own graph:

    torch.ops.ctclip.gemm_bf16(x, w, bias, residual)            # y = x @ w^T (+ bias) (+ residual)
    torch.ops.ctclip.layernorm(x, gamma, beta, eps)
    torch.ops.ctclip.cos_attn(q, k, v, q_scale, k_scale, heads, seq_len, layout, scale, bias, grid)
    torch.ops.ctclip.clip_infonce(text_latents, image_latents, log_temp)
    torch.ops.ctclip.vq_cos_argmax(x, codebook)                 # (idx int32, l2norm(x))
    torch.ops.ctclip.peg_dwconv3d(x, weight, bias, shape, mode)  # x + PEG(x), canonical rows
    torch.ops.ctclip.cpb_mlp(rel, w0, b0, w1, b1, w2, b2)        # CPB table [heads, bins]
    torch.ops.ctclip.patch_embed_i16(video, ln1_w, ln1_b, w, b, ln2_w, ln2_b, pt, p)   # to_patch_emb
    torch.ops.ctclip.bert_layer(x, attention_mask, heads, eps, wq, bq, ..., ln2_w, ln2_b)  # eval

Device tensors only (the ops are registered for the "cuda" device type, which is HIP on ROCm):
a CPU tensor raises, and with the library missing every op raises (``_lib.lib``).  Reference
call sites: ct_clip/attention.py:44-52,88-181 (linears, LayerNorm, cosine attention), :56-84
(PEG), :229-276 (continuous position bias),
ct_clip/ct_clip.py:796-812 (InfoNCE), ct_clip/ctvit.py:421-427 (VQ cosine argmax), :169-174
(patch embedding), ct_clip/ct_clip.py:685-686 (the BERT text tower's layers)."""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch
from torch import Tensor

from . import kernels as K

BF16 = torch.bfloat16
F32 = torch.float32


def _need(cond, msg):
    if not cond:
        raise ValueError(msg)


# ------------------------------------------------------------------------------ gemm_bf16
@torch.library.custom_op('ctclip::gemm_bf16', mutates_args=(), device_types='cuda')
def gemm_bf16(x: Tensor, w: Tensor, bias: Optional[Tensor] = None, residual: Optional[Tensor] = None) -> Tensor:
    """nn.Linear on the MFMA GEMM: x [M, K] bf16, w [N, K] bf16, bias [N] f32, residual [M, N] f32.
    Output bf16, or f32 when a residual is added (the residual stream is f32)."""
    _need(x.dtype == BF16 and w.dtype == BF16, 'gemm_bf16: x and w must be bf16')
    _need(x.dim() == 2 and w.dim() == 2 and x.shape[1] == w.shape[1], 'gemm_bf16: x [M, K], w [N, K]')
    _need(bias is None or (bias.dtype == F32 and bias.shape == (w.shape[0],)), 'gemm_bf16: bias [N] f32')
    _need(residual is None or (residual.dtype == F32 and residual.shape == (x.shape[0], w.shape[0])),
          'gemm_bf16: residual [M, N] f32')
    return K.linear(x.contiguous(), w.contiguous(), bias=bias,
                    residual=residual.contiguous() if residual is not None else None,
                    out_dtype=F32 if residual is not None else BF16)


@gemm_bf16.register_fake
def _(x, w, bias=None, residual=None):
    return x.new_empty(x.shape[0], w.shape[0], dtype=F32 if residual is not None else BF16)


def _gemm_setup(ctx, inputs, output):
    x, w, bias, residual = inputs
    ctx.save_for_backward(x, w)
    ctx.has_bias, ctx.has_res = bias is not None, residual is not None


def _gemm_bwd(ctx, dy):
    x, w = ctx.saved_tensors
    dyb = dy.to(BF16).contiguous()
    dx = K.matmul_nn(dyb, w.contiguous()) if ctx.needs_input_grad[0] else None
    dw = K.matmul_tn(dyb, x.contiguous()).to(w.dtype) if ctx.needs_input_grad[1] else None
    db = K.colsum(dy.contiguous()) if ctx.has_bias and ctx.needs_input_grad[2] else None
    dres = dy.to(F32) if ctx.has_res and ctx.needs_input_grad[3] else None
    return dx, dw, db, dres


gemm_bf16.register_autograd(_gemm_bwd, setup_context=_gemm_setup)


# ------------------------------------------------------------------------------ layernorm
@torch.library.custom_op('ctclip::layernorm', mutates_args=(), device_types='cuda')
def _layernorm(x: Tensor, gamma: Tensor, beta: Tensor, eps: float) -> Tuple[Tensor, Tensor, Tensor]:
    _need(x.dim() == 2 and x.dtype == F32, 'layernorm: x [rows, D] f32')
    _need(gamma.dtype == F32 and beta.dtype == F32 and gamma.shape == (x.shape[1],) == beta.shape,
          'layernorm: gamma / beta [D] f32')
    _, y, mean, rstd = K.layernorm_fwd(x.contiguous(), gamma, beta, eps, out_bf16=False, out_f32=True)
    return y, mean, rstd


@_layernorm.register_fake
def _(x, gamma, beta, eps):
    return x.new_empty(x.shape), x.new_empty(x.shape[0]), x.new_empty(x.shape[0])


def _ln_setup(ctx, inputs, output):
    x, gamma, _, _ = inputs
    _, mean, rstd = output
    ctx.save_for_backward(x, gamma, mean, rstd)


def _ln_bwd(ctx, dy, _dmean, _drstd):
    x, gamma, mean, rstd = ctx.saved_tensors
    dx, _, dg, db = K.layernorm_bwd(dy.contiguous(), x.contiguous(), mean, rstd, gamma, want_beta=True,
                                    dx_f32=True, dx_bf16=False)
    return dx, dg, db, None


_layernorm.register_autograd(_ln_bwd, setup_context=_ln_setup)


def layernorm(x: Tensor, gamma: Tensor, beta: Tensor, eps: float = 1e-5) -> Tensor:
    """LayerNorm over the last dim of x [rows, D] (f32 in / out); ct_clip/attention.py:28-35."""
    return _layernorm(x, gamma, beta, eps)[0]


# ------------------------------------------------------------------------------- cos_attn
@torch.library.custom_op('ctclip::cos_attn', mutates_args=(), device_types='cuda')
def _cos_attn(q: Tensor, k: Tensor, v: Tensor, q_scale: Tensor, k_scale: Tensor, heads: int, seq_len: int,
              layout: List[int], scale: float, bias: Optional[Tensor], grid: List[int]) -> Tuple[Tensor, Tensor]:
    M, HD = q.shape
    D = HD // heads
    _need(q.dtype == k.dtype == v.dtype == BF16 and k.shape == q.shape == v.shape, 'cos_attn: q / k / v [M, H*D] bf16')
    _need(D in (32, 64) and HD == heads * D, 'cos_attn: dim_head 32 or 64')
    _need(len(layout) == 4 and len(grid) == 2, 'cos_attn: layout (n_inner, s_outer, s_inner, s_pos), grid (h, w)')
    _need(M % seq_len == 0, 'cos_attn: rows must be a whole number of sequences')
    _need(bias is None or (bias.dtype == F32 and bias.dim() == 2 and bias.shape[0] == heads
                           and grid[0] * grid[1] == seq_len
                           and bias.shape[1] == (2 * grid[0] - 1) * (2 * grid[1] - 1)),
          'cos_attn: bias [heads, (2h-1)(2w-1)] f32 over an h x w grid of seq_len keys')
    qn = K.l2norm_scale_fwd(q.contiguous(), heads, D, q_scale)
    kn = K.l2norm_scale_fwd(k.contiguous(), heads, D, k_scale)
    o, lse = K.attn_fwd(qn, kn, v.contiguous(), L=seq_len, H=heads, D=D, nseq=M // seq_len, scale=scale,
                        seq=tuple(layout), bias_u=bias, grid=tuple(grid) if bias is not None else (0, 0))
    return o, lse


@_cos_attn.register_fake
def _(q, k, v, q_scale, k_scale, heads, seq_len, layout, scale, bias, grid):
    return q.new_empty(q.shape), q.new_empty(heads, q.shape[0], dtype=F32)


def _attn_setup(ctx, inputs, output):
    q, k, v, q_scale, k_scale, heads, seq_len, layout, scale, bias, grid = inputs
    o, lse = output
    ctx.save_for_backward(q, k, v, q_scale, k_scale, o, lse, bias)
    ctx.cfg = (heads, seq_len, tuple(layout), scale, tuple(grid), bias is not None)


def _attn_bwd(ctx, do, _dlse):
    q, k, v, q_scale, k_scale, o, lse, bias = ctx.saved_tensors
    heads, L, layout, scale, grid, has_bias = ctx.cfg
    M, HD = q.shape
    D = HD // heads
    q, k, v = q.contiguous(), k.contiguous(), v.contiguous()
    qn = K.l2norm_scale_fwd(q, heads, D, q_scale)
    kn = K.l2norm_scale_fwd(k, heads, D, k_scale)
    dqn, dkn, dv = torch.empty_like(qn), torch.empty_like(kn), torch.empty_like(v)
    du = torch.zeros_like(bias) if has_bias else None
    K.attn_bwd(qn, kn, v, o, lse, do.to(BF16).contiguous(), dqn, dkn, dv, L=L, H=heads, D=D, nseq=M // L,
               scale=scale, seq=layout, bias_u=bias if has_bias else None, dbias_u=du,
               grid=grid if has_bias else (0, 0))
    dq, dk = torch.empty_like(q), torch.empty_like(k)
    dqs = K.l2norm_scale_bwd(q, dqn, heads, D, q_scale, dq)
    dks = K.l2norm_scale_bwd(k, dkn, heads, D, k_scale, dk)
    return dq, dk, dv, dqs, dks, None, None, None, None, du, None


_cos_attn.register_autograd(_attn_bwd, setup_context=_attn_setup)


def cos_attn(q: Tensor, k: Tensor, v: Tensor, q_scale: Tensor, k_scale: Tensor, heads: int, seq_len: int,
             layout=None, scale: float = 8.0, bias: Optional[Tensor] = None, grid=(0, 0)) -> Tensor:
    """Cosine-similarity attention of ct_clip/attention.py:88-181: per head, q and k are
    l2-normalised and multiplied by the learned q_scale / k_scale [dim_head], sim = scale * q.k
    (+ the continuous position bias bias[h][bin(query, key)] over an h x w grid), softmax, . v.
    Rows [M, heads*dim_head] bf16; `layout` maps (sequence, position) to a row (default:
    contiguous sequences of seq_len rows; functional.Geo.seq gives the spatial / temporal ones)."""
    if layout is None:
        layout = (1, seq_len, 0, 1)
    return _cos_attn(q, k, v, q_scale, k_scale, heads, seq_len, list(layout), float(scale), bias, list(grid))[0]


# --------------------------------------------------------------------------- clip_infonce
@torch.library.custom_op('ctclip::clip_infonce', mutates_args=(), device_types='cuda')
def _clip_infonce(text_latents: Tensor, image_latents: Tensor, log_temp: Tensor) -> Tuple[Tensor, Tensor, Tensor,
                                                                                            Tensor]:
    _need(text_latents.dtype == image_latents.dtype == log_temp.dtype == F32, 'clip_infonce: f32 inputs')
    _need(text_latents.shape == image_latents.shape and text_latents.dim() == 2, 'clip_infonce: [B, dim_latent]')
    _need(log_temp.numel() == 1, 'clip_infonce: log_temp is a scalar')
    loss, dt, di, dlt, _, _, _ = K.clip_loss(text_latents.contiguous(), image_latents.contiguous(),
                                             log_temp.reshape(1).contiguous())
    return loss.reshape(()), dt, di, dlt.reshape(log_temp.shape)


@_clip_infonce.register_fake
def _(text_latents, image_latents, log_temp):
    return (text_latents.new_empty(()), torch.empty_like(text_latents), torch.empty_like(image_latents),
            torch.empty_like(log_temp))


def _clip_setup(ctx, inputs, output):
    _, dt, di, dlt = output
    ctx.save_for_backward(dt, di, dlt)


def _clip_bwd(ctx, dloss, *_):
    dt, di, dlt = ctx.saved_tensors
    return dt * dloss, di * dloss, dlt * dloss


_clip_infonce.register_autograd(_clip_bwd, setup_context=_clip_setup)


def clip_infonce(text_latents: Tensor, image_latents: Tensor, log_temp: Tensor) -> Tensor:
    """Symmetric InfoNCE of ct_clip/ct_clip.py:796-812 on raw latents: l2-normalise both, sim =
    exp(log_temp) * t . i^T, loss = (CE(sim, arange) + CE(sim^T, arange)) / 2 (scalar)."""
    return _clip_infonce(text_latents, image_latents, log_temp)[0]


# -------------------------------------------------------------------------- vq_cos_argmax
@torch.library.custom_op('ctclip::vq_cos_argmax', mutates_args=(), device_types='cuda')
def vq_cos_argmax(x: Tensor, codebook: Tensor) -> Tuple[Tensor, Tensor]:
    """Exact f32 cosine argmax of each row of x [M, D] against codebook [C, D] (f32 rows), as
    vector_quantize_pytorch's cosine codebook (ct_clip/ctvit.py:421-427): bf16 MFMA scores with a
    per-64-code-group (best, second-best) epilogue, then the f32 re-score of every code within the
    bf16 error margin.  Returns (indices int32 [M], l2norm(x) f32 [M, D])."""
    _need(x.dtype == F32 and codebook.dtype == F32 and x.dim() == 2 and codebook.dim() == 2
          and x.shape[1] == codebook.shape[1], 'vq_cos_argmax: x [M, D], codebook [C, D], f32')
    _need(x.shape[1] % 8 == 0, 'vq_cos_argmax: D % 8 == 0')
    x = x.contiguous()
    cb = codebook.contiguous()
    M, D = x.shape
    C = cb.shape[0]
    xn_b = K.l2norm_scale_fwd(K.cast_bf16(x), 1, D, torch.ones(D, device=x.device, dtype=F32))
    nt = (C + 63) // 64
    cand = torch.empty(M, nt, 2, device=x.device, dtype=F32)
    cand2 = torch.empty(M, nt, device=x.device, dtype=F32)
    K.gemm_raw(M, C, D, xn_b, D, True, K.cast_bf16(cb), D, True, cand, nt, C2=cand2, ldc2=nt, act=K.ACT_ARGMAX)
    idx, xn = K.vq_select(cand, x, cb, want_xn=True, cand2=cand2)
    return idx, xn


@vq_cos_argmax.register_fake
def _(x, codebook):
    return x.new_empty(x.shape[0], dtype=torch.int32), x.new_empty(x.shape)


# --------------------------------------------------------------------------- peg_dwconv3d
@torch.library.custom_op('ctclip::peg_dwconv3d', mutates_args=(), device_types='cuda')
def peg_dwconv3d(x: Tensor, weight: Tensor, bias: Tensor, shape: List[int], mode: int) -> Tensor:
    """x + PEG(x) (ct_clip/attention.py:56-84,324): depthwise 3x3x3 Conv3d, causal in time (pad
    (1, 1, 1, 1, 2, 0)), on token rows x [B*T*H*W, D] f32 in canonical (b, t, h, w) order.  mode 0:
    the spatial transformer's view; mode 1: the temporal transformer's raw-reshape view of its
    '(b h w) t d' tensor (attention.py:69-70).  weight [D, 1, 3, 3, 3] f32, bias [D] f32.  The
    conv reads the f32 x (as the model does since round 5, ctclip_peg_fwd_x32)."""
    B, T, H, W = shape
    D = x.shape[1]
    _need(x.dtype == F32 and x.dim() == 2 and x.shape[0] == B * T * H * W, 'peg_dwconv3d: x [B*T*H*W, D] f32')
    _need(weight.dtype == F32 and weight.numel() == D * 27 and bias.dtype == F32 and bias.shape == (D,),
          'peg_dwconv3d: weight [D, 1, 3, 3, 3], bias [D] f32')
    _need(mode in (0, 1), 'peg_dwconv3d: mode 0 (spatial) or 1 (temporal)')
    x = x.contiguous()
    outf, _, _, _, _ = K.peg_fwd_x32(x, B, T, H, W, weight.contiguous(), bias.contiguous(), mode)
    return outf


@peg_dwconv3d.register_fake
def _(x, weight, bias, shape, mode):
    return torch.empty_like(x)


def _peg_setup(ctx, inputs, output):
    x, weight, _, shape, mode = inputs
    ctx.save_for_backward(x, weight)
    ctx.cfg = (tuple(shape), mode)


def _peg_bwd(ctx, dy):
    x, weight = ctx.saved_tensors
    (B, T, H, W), mode = ctx.cfg
    dy = dy.contiguous()
    dxf, _, dw, db = K.peg_bwd(K.cast_bf16(dy), dy, K.cast_bf16(x.contiguous()), B, T, H, W,
                               weight.contiguous(), mode)
    return dxf, dw.reshape(weight.shape), db, None, None


peg_dwconv3d.register_autograd(_peg_bwd, setup_context=_peg_setup)


# -------------------------------------------------------------------------------- cpb_mlp
@torch.library.custom_op('ctclip::cpb_mlp', mutates_args=(), device_types='cuda')
def _cpb_mlp(rel: Tensor, w0: Tensor, b0: Tensor, w1: Tensor, b1: Tensor, w2: Tensor,
             b2: Tensor) -> Tuple[Tensor, Tensor, Tensor]:
    _need(all(t.dtype == F32 for t in (rel, w0, b0, w1, b1, w2, b2)), 'cpb_mlp: f32 tensors')
    _need(rel.dim() == 2 and rel.shape[1] == w0.shape[1] and w1.shape == (w0.shape[0], w0.shape[0])
          and w2.shape[1] == w0.shape[0], 'cpb_mlp: rel [bins, 2], w0 [d, 2], w1 [d, d], w2 [heads, d]')
    rel = rel.contiguous()
    nb, H = rel.shape[0], w2.shape[0]
    h1 = K.slinear(rel, w0.contiguous(), b0.contiguous(), act=1)
    h2 = K.slinear(h1, w1.contiguous(), b1.contiguous(), act=1)
    u = torch.empty(H, nb, device=rel.device, dtype=F32)
    w2 = w2.contiguous()
    K.sgemm(nb, H, h2.shape[1], h2, h2.stride(0), 1, w2, 1, w2.stride(0), u, 1, nb, bias=b2.contiguous())
    return u, h1, h2


@_cpb_mlp.register_fake
def _(rel, w0, b0, w1, b1, w2, b2):
    nb, d = rel.shape[0], w0.shape[0]
    return rel.new_empty(w2.shape[0], nb), rel.new_empty(nb, d), rel.new_empty(nb, d)


def _cpb_setup(ctx, inputs, output):
    rel, w0, _, w1, _, w2, _ = inputs
    _, h1, h2 = output
    ctx.save_for_backward(rel, w0, w1, w2, h1, h2)


def _cpb_bwd(ctx, du, _dh1, _dh2):
    rel, w0, w1, w2, h1, h2 = ctx.saved_tensors
    du = du.contiguous()
    H, nb = du.shape
    dev = du.device
    w0, w1, w2 = w0.contiguous(), w1.contiguous(), w2.contiguous()
    dz2 = torch.empty(nb, w2.shape[1], device=dev, dtype=F32)   # d(pre-activation of layer 2)
    K.sgemm(nb, w2.shape[1], H, du, 1, nb, w2, w2.stride(0), 1, dz2, dz2.stride(0), 1, act=2, aux=h2,
            sxm=h2.stride(0), sxn=1)
    dw2 = K.smm(du, h2)
    db2 = torch.empty(H, device=dev, dtype=F32)
    ones = torch.ones(nb, device=dev, dtype=F32)
    K.sgemm(H, 1, nb, du, nb, 1, ones, 1, 0, db2, 1, 1)
    dw1 = K.smm(dz2.t(), h1)
    db1 = K.colsum(dz2)
    dz1 = K.smm(dz2, w1, act=2, aux=h1)
    dw0 = K.smm(dz1.t(), rel.contiguous())
    db0 = K.colsum(dz1)
    drel = K.smm(dz1, w0) if ctx.needs_input_grad[0] else None
    return drel, dw0, db0, dw1, db1, dw2, db2


_cpb_mlp.register_autograd(_cpb_bwd, setup_context=_cpb_setup)


def cpb_mlp(rel: Tensor, w0: Tensor, b0: Tensor, w1: Tensor, b1: Tensor, w2: Tensor, b2: Tensor) -> Tensor:
    """ContinuousPositionBias's MLP (ct_clip/attention.py:229-276: Linear(2, d), LeakyReLU(0.1),
    Linear(d, d), LeakyReLU(0.1), Linear(d, heads)) on the distinct relative offsets rel [bins, 2]
    (functional.cpb_table: sign(x) log(|x| + 1) of the (dh, dw) offsets of an h x w grid).
    Returns the bias table [heads, bins] that cos_attn(bias=..., grid=(h, w)) consumes."""
    return _cpb_mlp(rel, w0, b0, w1, b1, w2, b2)[0]


# ------------------------------------------------------------------------ patch_embed_i16
@torch.library.custom_op('ctclip::patch_embed_i16', mutates_args=(), device_types='cuda')
def _patch_embed_i16(video: Tensor, ln1_w: Tensor, ln1_b: Tensor, w: Tensor, b: Tensor, ln2_w: Tensor,
                     ln2_b: Tensor, temporal_patch: int, patch: int) -> Tuple[Tensor, Tensor, Tensor, Tensor, Tensor]:
    from .layers import patch_offsets
    _need(video.dim() == 5 and video.dtype in (torch.int16, F32), 'patch_embed_i16: video [B, C, F, H, W] int16 / f32')
    Bv, C, Fr, H, W = video.shape
    PT, P = temporal_patch, patch
    _need(Fr % PT == 0 and H % P == 0 and W % P == 0, 'patch_embed_i16: frames / sides divisible by the patch')
    pd, dim = C * PT * P * P, w.shape[0]
    _need(w.dtype == F32 and w.shape == (dim, pd) and b.shape == (dim,) and ln1_w.shape == (pd,) == ln1_b.shape
          and ln2_w.shape == (dim,) == ln2_b.shape, 'patch_embed_i16: w [dim, c*pt*p*p], b / ln2 [dim], ln1 [pd]')
    video = video.contiguous()
    offs = patch_offsets(C, PT, P, P, H, W).to(video.device)
    kp = (pd + 63) // 64 * 64
    xhat_p = K.patch_ln(video, video.dtype == torch.int16, PT, P, offs, ld=kp)   # [M, kp] bf16
    Wp = K.pack_rows(w.contiguous(), dim, kp, colscale=ln1_w.contiguous())         # W diag(g1), bf16
    bp = K.slinear(ln1_b.view(1, -1), w, bias=b).view(-1)                          # b + W beta1
    y1 = K.linear(xhat_p, Wp, bias=bp, out_dtype=F32)
    _, yf, mean, rstd = K.layernorm_fwd(y1, ln2_w.contiguous(), ln2_b.contiguous(), 1e-5, out_bf16=False,
                                        out_f32=True)
    return yf, xhat_p, y1, mean, rstd


@_patch_embed_i16.register_fake
def _(video, ln1_w, ln1_b, w, b, ln2_w, ln2_b, temporal_patch, patch):
    Bv, C, Fr, H, W = video.shape
    M = Bv * (Fr // temporal_patch) * (H // patch) * (W // patch)
    kp = (w.shape[1] + 63) // 64 * 64
    return (w.new_empty(M, w.shape[0]), w.new_empty(M, kp, dtype=BF16), w.new_empty(M, w.shape[0]),
            w.new_empty(M), w.new_empty(M))


def _pe_setup(ctx, inputs, output):
    _, ln1_w, ln1_b, w, _, ln2_w, _, _, _ = inputs
    _, xhat_p, y1, mean, rstd = output
    ctx.save_for_backward(xhat_p, y1, mean, rstd, ln1_w, ln1_b, w, ln2_w)


def _pe_bwd(ctx, dy, *_):
    xhat_p, y1, mean, rstd, ln1_w, ln1_b, w, ln2_w = ctx.saved_tensors
    pd = w.shape[1]
    _, dy1b, dg2, db2 = K.layernorm_bwd(dy.contiguous(), y1, mean, rstd, ln2_w, dx_f32=False)
    G = K.matmul_tn(dy1b, xhat_p[:, :pd])                   # dy1^T xhat [dim, pd]
    cs = K.colsum(dy1b)                                      # d bias
    dw, dg1, db1 = torch.zeros_like(w), torch.zeros_like(ln1_w), torch.zeros_like(ln1_b)
    K.patch_wgrad(G, cs, w.contiguous(), ln1_w.contiguous(), ln1_b.contiguous(), dw, dg1, db1, accumulate=True)
    return None, dg1, db1, dw, cs, dg2, db2, None, None


_patch_embed_i16.register_autograd(_pe_bwd, setup_context=_pe_setup)


def patch_embed_i16(video: Tensor, ln1_w: Tensor, ln1_b: Tensor, w: Tensor, b: Tensor, ln2_w: Tensor,
                    ln2_b: Tensor, temporal_patch: int = 10, patch: int = 20) -> Tensor:
    """CTViT.to_patch_emb (ct_clip/ctvit.py:169-174: Rearrange 'b c (t pt) (h p1) (w p2) -> b t h w
    (c pt p1 p2)', LayerNorm(pd), Linear(pd, dim), LayerNorm(dim)) on the raw int16 HU volume, the
    input normalisation of ct_clip/data.py:150-152 fused (an f32 volume in [-1, 1] is taken as is).
    Returns the tokens [B*T*Hg*Wg, dim] f32 in canonical (b, t, h, w) order; differentiable in the
    weights (the volume is data)."""
    return _patch_embed_i16(video, ln1_w, ln1_b, w, b, ln2_w, ln2_b, temporal_patch, patch)[0]


# ----------------------------------------------------------------------------- bert_layer
class _NoCtx:
    """Stand-in autograd context for running a fused Function's forward as a plain op."""

    def save_for_backward(self, *_):
        pass

    def mark_non_differentiable(self, *_):
        pass

    def set_materialize_grads(self, *_):
        pass


@torch.library.custom_op('ctclip::bert_layer', mutates_args=(), device_types='cuda')
def bert_layer(x: Tensor, attention_mask: Tensor, heads: int, eps: float, wq: Tensor, bq: Tensor, wk: Tensor,
               bk: Tensor, wv: Tensor, bv: Tensor, wo: Tensor, bo: Tensor, ln1_w: Tensor, ln1_b: Tensor, wi: Tensor,
               bi: Tensor, wout: Tensor, bout: Tensor, ln2_w: Tensor, ln2_b: Tensor) -> Tensor:
    """transformers' BertLayer forward in eval mode (ct_clip/ct_clip.py:685-686 runs BERT-base; no
    dropout): x [B, L, hidden] f32, attention_mask [B, L] (1 = attend); the fused QKV GEMM (hi / lo
    split weights), the MFMA attention with the additive key mask, dense + residual + LayerNorm, GELU
    MLP, dense + residual + LayerNorm -- the kernels of functional.BertLayerFn, whose autograd form
    the model trains with.  Returns [B, L, hidden] f32."""
    from . import functional as Fn
    _need(x.dim() == 3 and x.dtype == F32, 'bert_layer: x [B, L, hidden] f32')
    B, L, Hd = x.shape
    _need(attention_mask.shape == (B, L), 'bert_layer: attention_mask [B, L]')
    _need(Hd % heads == 0 and Hd // heads in (32, 64), 'bert_layer: head dim 32 or 64')
    xf = x.reshape(B * L, Hd).contiguous()
    kmask = attention_mask.to(torch.int32).contiguous()
    ps = [t.detach().contiguous() for t in (wq, bq, wk, bk, wv, bv, wo, bo, ln1_w, ln1_b, wi, bi, wout, bout,
                                              ln2_w, ln2_b)]
    x2f, _ = Fn.BertLayerFn.forward(_NoCtx(), xf, K.cast_bf16(xf), kmask, B, L, heads, eps, *ps)
    return x2f.view(B, L, Hd)


@bert_layer.register_fake
def _(x, attention_mask, heads, eps, *ws):
    return torch.empty_like(x)
