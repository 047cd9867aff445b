"""Opt-in f32 image tower: the 3D-ViT forward (and the image projection) with f32 activations and
exact-f32 products, for outputs that must match the reference's fp32 run index for index.

The reference computes the whole step in fp32 (``accelerator.autocast()`` is a no-op with empty
``accelerate_kwargs``, ct_clip/CTCLIPTrainer.py:210,216,342).  The default image tower runs its
GEMMs and attention on bf16 operands (~1e-2 relative token error before the VQ), which flips the
cosine argmax of ct_clip/ctvit.py:427 on ~2 % of tokens whose top-2 margin is small (SURVEY 8(c)
counts only flips below a 1e-6 margin as ties).  ``set_vit_precision('f32')`` switches the
tower's forward to:

  * patchify + LayerNorm(4000) in f32 (``ctclip_patch_ln_f32``), then ``to_patch_emb``'s Linear
    and LayerNorm(512) in f32 (ctvit.py:169-174);
  * per layer: PEG (``ctclip_peg_fwd_f32``), bias-less LN, to_q / to_kv, l2norm * scale, cosine
    attention with the CPB bias (``ctclip_attn_fwd_f32``), to_out + residual, FF LayerNorm,
    FF1, GEGLU, FF2 + residual (attention.py:56-84,127-181,39-52,311-333); norm_out;
  * every Linear on ``ctclip_sgemm`` (v_mfma_f32_16x16x4_f32: an f32 fma chain per output);
  * the VQ unchanged (its f32 re-score already returns the exact f32 argmax of its input tokens);
  * the 294,912-wide ``to_visual_latent`` in f32 as well.

Forward only (the bf16 kernels own the training backward): calling it with autograd recording a
graph through trainable tower weights raises.  Cost: DESIGN.md §5 (measured forward time)."""
from __future__ import annotations

import torch

from . import kernels as K

F32 = torch.float32
_MODE = {'vit': 'bf16'}


def set_vit_precision(mode):
    """'bf16' (default: bf16 MFMA kernels, forward + backward) or 'f32' (forward-only exact-f32
    image tower).  Returns the previous mode."""
    if mode not in ('bf16', 'f32'):
        raise ValueError(mode)
    old = _MODE['vit']
    _MODE['vit'] = mode
    return old


def vit_precision():
    return _MODE['vit']


def _check_no_grad(module):
    if torch.is_grad_enabled() and any(p.requires_grad for p in module.parameters()):
        raise NotImplementedError("the f32 image tower is forward-only: call it under torch.no_grad() or "
                                  "with frozen weights (set_vit_precision('bf16') for training)")


def _ln(x, gamma, beta, eps=1e-5):
    return K.layernorm_fwd(x, gamma, beta, eps, out_bf16=False, out_f32=True)[1]


def _linear(x, W, bias=None, residual=None):
    """x [M, K] f32 @ W[N, K]^T (+bias) (+residual), exact f32 (ctclip_sgemm)."""
    if residual is not None:
        out = residual.clone()
        return K.slinear(x, W.detach(), bias=bias, out=out, accumulate=True)
    return K.slinear(x, W.detach(), bias=bias)


def vit_layer_f32(x, geo, bias_u, peg, attn, ff):
    """One CTViT transformer layer (ct_clip/attention.py:322-331) in f32: x = PEG(x) + x;
    x = Attention(x, bias) + x; x = FeedForward(x) + x."""
    H, dh = geo.heads, geo.dim_head
    inner = H * dh
    x1 = K.peg_fwd_f32(x, geo.B, geo.T, geo.Hg, geo.Wg, peg.dsconv.weight.detach(), peg.dsconv.bias.detach(),
                       geo.mode)
    xn = _ln(x1, attn.norm.gamma.detach(), None)                       # attention.py:139-141 (q side only)
    q = _linear(xn, attn.to_q.weight)
    kv = _linear(x1, attn.to_kv.weight)                                # K / V from the un-normalised x
    qn = K.l2norm_scale_fwd_f32(q, H, dh, attn.q_scale.detach())
    kn = K.l2norm_scale_fwd_f32(kv[:, :inner], H, dh, attn.k_scale.detach())
    L, nseq, seq = geo.seq()
    use_bias = bias_u is not None
    o = K.attn_fwd_f32(qn, kn, kv[:, inner:], L=L, H=H, D=dh, nseq=nseq, scale=8.0, seq=seq,
                       bias_u=bias_u if use_bias else None, grid=(geo.Hg, geo.Wg) if use_bias else (0, 0))
    x2 = _linear(o, attn.to_out.weight, residual=x1)
    xn2 = _ln(x2, ff[0].weight.detach(), ff[0].bias.detach())
    h = _linear(xn2, ff[1].weight)                                     # [M, 2 * inner_ff]: x | gate
    g = K.geglu_f32(h)
    return _linear(g, ff[4].weight, residual=x2)


def encode_tokens_f32(vt, video, trace=None):
    """``CTViT.encode_tokens`` in f32 (see module docstring): (z f32 [M, D], z bf16, geometry)."""
    from . import functional as Fn
    _check_no_grad(vt)
    if video.ndim == 4:
        video = video.unsqueeze(2)
    B, C, F, H, W = video.shape
    assert (H, W) == tuple(vt.image_size), (H, W)
    is_hu = video.dtype == torch.int16
    if not is_hu and video.dtype != F32:
        video = video.float()
    video = video.contiguous()
    pe = vt.to_patch_emb
    PT, P = vt.temporal_patch_size, vt.patch_size[0]
    xn0 = K.patch_ln_f32(video, is_hu, PT, P, vt._offsets(video.shape, video.device), pe[1].weight.detach(),
                         pe[1].bias.detach())
    y1 = _linear(xn0, pe[2].weight, bias=pe[2].bias.detach())
    del xn0
    x = _ln(y1, pe[3].weight.detach(), pe[3].bias.detach())
    if trace is not None:
        trace['patch_emb'] = x
    hg, wg = vt.patch_height_width
    T = F // PT
    g_sp = Fn.Geo(B, T, hg, wg, vt.heads, vt.dim_head, 0)
    g_tm = Fn.Geo(B, T, hg, wg, vt.heads, vt.dim_head, 1)
    with torch.no_grad():
        bias_u = vt.spatial_rel_pos_bias(hg, wg)                       # f32 already (CPBFn, sgemm)
    for peg, attn, _, ff in vt.enc_spatial_transformer.layers:
        x = vit_layer_f32(x, g_sp, bias_u, peg, attn, ff)
    x = _ln(x, vt.enc_spatial_transformer.norm_out.gamma.detach(), None)
    if trace is not None:
        trace['spatial_out'] = x
    for peg, attn, _, ff in vt.enc_temporal_transformer.layers:
        x = vit_layer_f32(x, g_tm, None, peg, attn, ff)
    z = _ln(x, vt.enc_temporal_transformer.norm_out.gamma.detach(), None)
    if trace is not None:
        trace['temporal_out'] = z
    return z, K.cast_bf16(z), g_sp


def project_f32(W, pooled):
    """``to_visual_latent`` (ct_clip/ct_clip.py:564,767) in exact f32: [B, 294912] @ W^T."""
    return K.slinear(pooled.contiguous(), W.detach())
