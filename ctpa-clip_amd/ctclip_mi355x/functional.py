"""Layer-level autograd Functions: each forward runs a fixed chain of HIP kernels and saves
what its hand-written backward needs.  No torch math on the hot path — torch provides device
memory, streams, autograd plumbing and RCCL collectives.

Data layout: the CTViT residual stream lives in canonical token order
(b, t, h, w) as an f32 master [M, D] plus a bf16 shadow for the GEMMs; the spatial and
temporal transformers address the same rows (attention / PEG kernels gather sequences
by index arithmetic instead of transposing).
"""
from __future__ import annotations

import math
import os
import weakref
from dataclasses import dataclass

import torch

from . import dist_sync
from . import kernels as K
from . import streams

F32, BF16 = torch.float32, torch.bfloat16


# ----------------------------------------------------------------------------- gradient plumbing
def gsink(p):
    """Gradient sink of parameter ``p``: the backward kernels accumulate its gradient straight
    into ``p.grad`` (the trainer binds every .grad to one flat f32 arena, zeroed after each
    optimizer step) and the Function returns None for ``p`` -- no temporary gradient and no
    AccumulateGrad add per parameter.  None when ``p`` needs no gradient."""
    if not p.requires_grad:
        return None
    if p.grad is None:
        p.grad = torch.zeros_like(p, memory_format=torch.contiguous_format)
    return p.grad


def gsink_cat(ps):
    """One gradient sink for parameters ``ps`` that sit consecutively, in order, in the trainer's
    arena (BERT's q / k / v weights, and their biases: bert.BertModel.param_order): a view of the
    gradient arena covering all of them, so one weight-gradient GEMM and one column sum serve the
    fused QKV projection.  None when they are not adjacent there or a .grad was rebound."""
    if not all(p.requires_grad for p in ps):
        return None
    a = _adjacent(ps, lambda f: f.grad)
    if a is None:
        return None
    arena, lo, hi = a
    if any(p.grad is None or p.grad.data_ptr() != arena[p._ctclip_off:].data_ptr() for p in ps):
        return None
    return arena[lo:hi].view(-1, *ps[0].shape[1:])


_SHADOW = {}


def put_shadow(gf, gb):
    """Register ``gb`` (bf16) as the bf16 image of the f32 gradient ``gf`` a backward returns,
    so the producing layer's backward can take it instead of re-casting (identity-checked)."""
    _SHADOW[id(gf)] = (weakref.ref(gf), gb)


def take_shadow(gf):
    e = _SHADOW.pop(id(gf), None)
    if e is not None and e[0]() is gf:
        return e[1]
    return None


def precise_f32():
    """True in the f32 image-tower mode (precise.set_vit_precision('f32')): the 3D-ViT Functions
    below then run their forward in exact f32 and save the bf16 tensors their backward kernels read,
    so the mode trains (f32 forward, bf16 backward)."""
    from . import precise
    return precise.vit_precision() == 'f32'


def precise_split():
    """True in the split-fp16 image-tower mode (precise.set_vit_precision('split'), round 6): the
    forward's Linears on the x3 GEMM (~22-bit operands, f32 accumulation), everything else in f32 --
    the f32 mode's numerics at a fraction of its cost; the backward as in the other modes."""
    from . import precise
    return precise.vit_precision() == 'split'


def x3_weight(W, rows=None, cols=None, rowmap=None, colscale=None, tag='w'):
    """Split-fp16 pair of f32 weight W for the x3 GEMM (kernels.pack_rows_x3, scaled by X3_WSCALE),
    cached on the parameter until the master changes (optimizer epoch, version, storage)."""
    key = (K.weights_epoch(), W._version, W.data_ptr(),
           None if colscale is None else (colscale.data_ptr(), colscale._version))
    cache = W.__dict__.setdefault('_ctclip_x3', {})
    e = cache.get(tag)
    if e is None or e[0] != key:
        e = (key, K.pack_rows_x3(W.detach(), rows or W.shape[0], cols or W.shape[1], rowmap=rowmap,
                                 colscale=None if colscale is None else colscale.detach()))
        cache[tag] = e
    return e[1]


# ----------------------------------------------------------------------------- geometry
@dataclass(frozen=True)
class Geo:
    B: int
    T: int
    Hg: int
    Wg: int
    heads: int
    dim_head: int
    mode: int            # 0 spatial transformer, 1 temporal transformer

    @property
    def M(self):
        return self.B * self.T * self.Hg * self.Wg

    def seq(self):
        """(L, nseq, (n_inner, s_outer, s_inner, s_pos)) for the attention row gather."""
        hw = self.Hg * self.Wg
        if self.mode == 0:     # '(b t) (h w) d'  (ct_clip/ctvit.py:315)
            return hw, self.B * self.T, (1, hw, 0, 1)
        # '(b h w) t d'  (ct_clip/ctvit.py:325): s = b*hw + j, row = b*T*hw + t*hw + j
        return self.T, self.B * hw, (hw, self.T * hw, 1, hw)


# ----------------------------------------------------------------------------- weight packing
_MAP_CACHE = {}


def ff_pad(inner):
    return (inner + 63) // 64 * 64


def ff1_rowmap(inner, device):
    """Row map of the GEGLU-interleaved W1: packed row t*64 + c  <- x row t*32+c,
    t*64 + 32 + c <- gate row inner + t*32 + c  (-1 = zero padding); 32-column pairs so one
    wave's 64 output columns always hold matching x / gate halves."""
    key = ('ff1', inner, str(device))
    if key not in _MAP_CACHE:
        P = ff_pad(inner)
        m = torch.full((2 * P,), -1, dtype=torch.int32)
        for t in range(P // 32):
            for c in range(32):
                j = t * 32 + c
                if j < inner:
                    m[t * 64 + c] = j
                    m[t * 64 + 32 + c] = inner + j
        _MAP_CACHE[key] = m.to(device)
    return _MAP_CACHE[key]


# packed FeedForward weights made ahead of the layers (prepack_ff, on the auxiliary stream at the
# start of the image tower's forward), keyed by the weight's storage, version and optimizer epoch
_PREPACKED = {}


def _pack_key(kind, W):
    return (kind, W.data_ptr(), W._version, K.weights_epoch())


def pack_ff1(W1):
    hit = _PREPACKED.get(_pack_key('ff1', W1))
    if hit is not None:
        return hit
    inner = W1.shape[0] // 2
    P = ff_pad(inner)
    return K.pack_rows(W1, 2 * P, W1.shape[1], rowmap=ff1_rowmap(inner, W1.device))


def pack_ff2(W2):
    hit = _PREPACKED.get(_pack_key('ff2', W2))
    if hit is not None:
        return hit
    return K.pack_rows(W2, W2.shape[0], ff_pad(W2.shape[1]))


def pack_ff1_h16(W1):
    """fp16 image of the GEGLU-interleaved W1 (the fp16 forward FF1 GEMM; pack_ff1 layout)."""
    hit = _PREPACKED.get(_pack_key('ff1h', W1))
    if hit is not None:
        return hit
    inner = W1.shape[0] // 2
    P = ff_pad(inner)
    return K.pack_rows_h16(W1, 2 * P, W1.shape[1], rowmap=ff1_rowmap(inner, W1.device))


def h16(W):
    """fp16 copy of an f32 weight (the fp16 forward GEMMs), cached by prepack_ff."""
    hit = _PREPACKED.get(_pack_key('h16', W))
    if hit is not None:
        return hit
    return K.pack_rows_h16(W, W.shape[0], W.shape[1])


def _fold_key(kind, Wq, gamma, Wkv, qs, ks):
    return (kind,) + tuple((t.data_ptr(), t._version) for t in (Wq, gamma, Wkv, qs, ks)) + (K.weights_epoch(),)


def qkv_fold_pack(Wq, gamma, Wkv, Wkv_b, q_scale, k_scale):
    """K.pack_qkv_fold of a layer (bf16 [Wq o gamma ; Wkv], fold sums, scales), prepacked by
    prepack_ff when the weights have not changed since."""
    hit = _PREPACKED.get(_fold_key('qkvf', Wq, gamma, Wkv, q_scale, k_scale))
    if hit is not None:
        return hit
    return K.pack_qkv_fold(Wq.detach(), gamma, Wkv_b, q_scale.detach(), k_scale.detach())


def qkv_fold_pack_h16(Wq, gamma, Wkv, q_scale, k_scale):
    """K.pack_qkv_fold_h16 of a layer (the fp16 forward's folded B operand and fold sums)."""
    hit = _PREPACKED.get(_fold_key('qkvh', Wq, gamma, Wkv, q_scale, k_scale))
    if hit is not None:
        return hit
    return K.pack_qkv_fold_h16(Wq.detach(), gamma, Wkv.detach())


def prepack_ff(pairs, wo=(), qkv=()):
    """Pack every layer's FeedForward weights now (on the caller's current stream) for the layers
    that run later (pack_ff1 / pack_ff2 then return these) -- with the fp16 forward also the fp16 W1
    images and the attention output weights `wo` -- and, for the LayerNorm-folded Q | K | V
    projection, each layer's folded B operand (`qkv`: (Wq, gamma, Wkv, q_scale, k_scale) per
    layer); returns the packed tensors."""
    _PREPACKED.clear()
    out = []
    for Wq, gamma, Wkv, qs, ks in qkv:
        f = K.pack_qkv_fold(Wq.detach(), gamma, bf(Wkv), qs.detach(), ks.detach())
        _PREPACKED[_fold_key('qkvf', Wq, gamma, Wkv, qs, ks)] = f
        out += list(f)
        if vit_f16():
            h = K.pack_qkv_fold_h16(Wq.detach(), gamma, Wkv.detach())
            _PREPACKED[_fold_key('qkvh', Wq, gamma, Wkv, qs, ks)] = h
            out += list(h)
    for W1, W2 in pairs:
        a, b = pack_ff1(W1), pack_ff2(W2)
        _PREPACKED[_pack_key('ff1', W1)] = a
        _PREPACKED[_pack_key('ff2', W2)] = b
        out += [a, b]
        if vit_f16():
            c = pack_ff1_h16(W1)
            _PREPACKED[_pack_key('ff1h', W1)] = c
            out.append(c)
    if vit_f16():
        for W in wo:
            c = h16(W)
            _PREPACKED[_pack_key('h16', W)] = c
            out.append(c)
    return out


def shadow_bf16(W):
    """The bf16 copy of parameter W that the trainer's Adam kernel keeps (trainer.FlatParams), or
    None when W has none or was changed since it was written."""
    sh = getattr(W, '_ctclip_bf16', None)
    if sh is None or W._version != getattr(W, '_ctclip_ver', -1) or W.data_ptr() != getattr(W, '_ctclip_ptr', 0):
        return None
    return sh


def bf(W):
    """bf16 weight for the MFMA GEMMs: the Adam-maintained shadow when current, else a cast."""
    sh = shadow_bf16(W)
    return sh if sh is not None else K.cast_bf16(W.contiguous())


# The text tower's forward GEMMs read each weight as W = hi + lo (two bf16 images, ~16 mantissa
# bits; gemm.hip walks K twice into one f32 accumulator): the bf16 rounding of BERT-base's weights
# is what put its latents 1.4e-3 off the f32 reference (tools/bert_precision.py: 6e-4 without
# it).  CTCLIP_TEXT_SPLIT=0 restores single bf16 weights (A/B switch).
_TEXT_SPLIT = os.environ.get('CTCLIP_TEXT_SPLIT', '1') != '0'
# hi / lo split weights on the top CTCLIP_TEXT_SPLIT_LAYERS BERT layers only (default: all 12)
_TEXT_SPLIT_LAYERS = int(os.environ.get('CTCLIP_TEXT_SPLIT_LAYERS', '1000'))
# BERT hidden dropout folded into the split-K combine (forward) and the LayerNorm backward, the
# GELU backward into the dX GEMM (act 6), the dense bias gradients into the LayerNorm backward's
# partials; CTCLIP_BERT_FUSE=0 restores the stand-alone dropout / gelu_bwd / colsum kernels (A/B)
_BERT_FUSE = os.environ.get('CTCLIP_BERT_FUSE', '1') != '0'
# A/B only: the FeedForward's K = 2,816 dX GEMM (a plain bf16 output) on hipBLASLt via torch.matmul
_DXN2_BLAS = os.environ.get('CTCLIP_DXN2_BLAS', '0') != '0'


def bf_split(W):
    """(hi, lo) bf16 images of f32 weight W: the Adam-maintained shadows when current, else a split cast."""
    sh = shadow_bf16(W)
    lo = getattr(W, '_ctclip_bf16_lo', None)
    if sh is not None and lo is not None:
        return sh, lo
    return K.cast_bf16_split(W.detach().contiguous())


def bf_cat_split(ws):
    """bf_split of torch.cat(ws, 0): views of the shadow arenas when the weights are adjacent there."""
    if all(shadow_bf16(w) is not None and getattr(w, '_ctclip_bf16_lo', None) is not None for w in ws):
        a = _adjacent(ws, lambda f: f.bf16)
        if a is not None:
            arena, lo, hi = a
            shp = (-1, *ws[0].shape[1:])
            return arena[lo:hi].view(shp), ws[0]._ctclip_flat.bf16_lo[lo:hi].view(shp)
    return K.cast_bf16_split(torch.cat([w.detach() for w in ws], 0).contiguous())


def _adjacent(ts, arena_of):
    """(arena, first offset) when tensors ts are consecutive, in order, in one arena."""
    flat = getattr(ts[0], '_ctclip_flat', None)
    if flat is None or any(getattr(t, '_ctclip_flat', None) is not flat for t in ts):
        return None
    off = ts[0]._ctclip_off
    o = off
    for t in ts:
        if t._ctclip_off != o:
            return None
        o += t.numel()
    return arena_of(flat), off, o


# ----------------------------------------------------------------------------- MX-fp8 (configs[3])
# The 3D-ViT's five forward linears (Q, KV, attention out, FF1 + GEGLU, FF2) run as MX-fp8 GEMMs
# (csrc/mxfp8.hip: e4m3 elements, one e8m0 scale per 32 k) when enabled: activations quantised per
# call, weights once per optimizer update.  The backward stays bf16 on the same saved bf16
# activations and weights.  SURVEY 8(c): compared to the build's own bf16 path, tolerance per test.
_FP8 = {'on': False}
_L2N_FUSED = os.environ.get('CTCLIP_L2N_FUSED', '1') != '0'   # A/B switch of the act-5 projections
# The attention's pre-norm LayerNorm folded into ONE Q | K | V projection over the PEG output
# (gemm256.hip EP 8, ctclip_gemm_qkv_lnfold): PEG leaves the LayerNorm statistics, the Q columns
# compute LN(x) Wq^T = rstd (x (gamma o Wq)^T - mean Wq gamma), so neither the LayerNorm kernel
# nor its output exists; the Q weight gradient uses the same fold (ctclip_lnfold_wgrad).
# CTCLIP_LN1_FOLD=0: the LayerNorm kernel and the two projections (A/B switch).
_LN1_FOLD = os.environ.get('CTCLIP_LN1_FOLD', '1') != '0'
# the FeedForward weight gradients' split-K slabs reduced straight into the unpacked .grad rows
# (ctclip_reduce_slabs_rows); CTCLIP_DW_UNPACK_FUSED=0: slab reduction + unpack_rows (A/B)
_DW_UNPACK_FUSED = os.environ.get('CTCLIP_DW_UNPACK_FUSED', '1') != '0'
# the training VQ's EMA statistics accumulated in code-sorted order (kernels.vq_ema_accum with a work
# buffer: ~10x fewer int64 atomics than the token-order kernel, same sums bit for bit);
# CTCLIP_VQ_EMA_SORTED=0: token order (A/B)
_EMA_SORTED = os.environ.get('CTCLIP_VQ_EMA_SORTED', '1') != '0'
# fold backward: the q and k l2norm backwards as one pass (ctclip_l2norm_qk_bwd_fold); 0 = two (A/B)
_QK_BWD_MERGED = os.environ.get('CTCLIP_QK_BWD_MERGED', '1') != '0'
_QKV_WGRAD = os.environ.get('CTCLIP_QKV_WGRAD', '1') != '0'   # A/B switch of BERT's merged q/k/v wgrad
# PEG forward taps from the f32 residual stream instead of its bf16 shadow (ctclip_peg_fwd_x32, round 5:
# the shadow's rounding was ~22 % of the bf16 tower's squared pre-VQ error, tools/vit_precision.py);
# CTCLIP_PEG_X32=0: the bf16-tap kernel (A/B)
_PEG_X32 = os.environ.get('CTCLIP_PEG_X32', '1') != '0'
# The 3D-ViT forward GEMMs -- patch embedding, the LayerNorm-folded Q | K | V projection, to_out (+ the
# FeedForward LayerNorm) and FF1 -- on fp16 operands (round 5): fp16 has 3 more mantissa bits than
# bf16 at the same MFMA rate, and these operands (LayerNorm outputs, the residual stream, unit-norm
# attention outputs, weights ~1e-2) sit well inside its range.  The producers write an fp16 copy beside
# the bf16 tensor the backward reads (the backward stays bf16); FF1's h is stored in fp16 (the GEGLU
# backward reads it).  tools/vit_precision.py: pre-VQ token error 1.05e-2 -> ~4e-3 with the f32-tap
# PEG.  CTCLIP_VIT_F16=0: the bf16 forward (A/B).
_VIT_F16 = {'on': os.environ.get('CTCLIP_VIT_F16', '1') != '0'}


def vit_f16():
    return _VIT_F16['on']


def set_vit_f16(on):
    """Switch the fp16 forward GEMMs of the 3D-ViT on / off; returns the previous setting."""
    old = _VIT_F16['on']
    _VIT_F16['on'] = bool(on)
    return old


# image projection forward on the skinny streaming GEMM (ctclip_skinny_gemm); 0 = split-K tile (A/B)
_SKINNY_PROJ = os.environ.get('CTCLIP_SKINNY_PROJ', '1') != '0'


def set_vit_fp8(on):
    """Switch the 3D-ViT forward linears to MX-fp8 (True) or bf16 (False); returns the previous."""
    old = _FP8['on']
    _FP8['on'] = bool(on)
    return old


def vit_fp8():
    return _FP8['on']


def fp8_weight(W, tag, Wb):
    """(q, scales) of the bf16 weight image Wb of parameter W, cached ON the parameter and
    re-quantised whenever the master changed: an optimizer update (weights_epoch; Adam writes the
    arena through raw pointers), an in-place copy / load_state_dict (W._version) or a re-bound
    storage (data_ptr).  Dies with the parameter (no module-level cache keeping dead models alive)."""
    key = (K.weights_epoch(), W._version, W.data_ptr())
    cache = W.__dict__.setdefault('_ctclip_fp8', {})
    e = cache.get(tag)
    if e is None or e[0] != key:
        e = (key,) + K.quant_mxfp8(Wb)
        cache[tag] = e
    return e[1], e[2]


def fp8_linear(x, W, tag, Wb, **kw):
    """x[M, K] (bf16) @ Wb[N, K]^T through the MX-fp8 GEMM (epilogue keywords of gemm_mxfp8);
    Wb is the bf16 (packed) image of parameter W."""
    qa, sa = K.quant_mxfp8(x)
    qb, sb = fp8_weight(W, tag, Wb)
    return K.gemm_mxfp8(qa, sa, qb, sb, **kw)


def bf_cat(ws):
    """bf16 of torch.cat(ws, 0): a view of the shadow arena when the weights are adjacent there
    (BERT's q / k / v, see bert.BertModel.param_order), else cat + cast."""
    if all(shadow_bf16(w) is not None for w in ws):
        a = _adjacent(ws, lambda f: f.bf16)
        if a is not None:
            arena, lo, hi = a
            return arena[lo:hi].view(-1, *ws[0].shape[1:])
    return K.cast_bf16(torch.cat(ws, 0))


def cat_f32(ts):
    """torch.cat(ts, 0) of f32 parameters: a view of the parameter arena when adjacent there."""
    a = _adjacent(ts, lambda f: f.data)
    if a is not None and all(t.data_ptr() == getattr(t, '_ctclip_ptr', 0) for t in ts):
        arena, lo, hi = a
        return arena[lo:hi].view(-1, *ts[0].shape[1:])
    return torch.cat(ts, 0).contiguous()


# ----------------------------------------------------------------------------- patch embedding
class PatchEmbedFn(torch.autograd.Function):
    """``CTViT.to_patch_emb`` (ct_clip/ctvit.py:169-174) with the input normalisation of
    ct_clip/data.py:150-152 fused when the volume arrives as int16 HU.
    LayerNorm(patch) affine is folded into the Linear: W' = W diag(g), b' = b + W beta."""

    @staticmethod
    def forward(ctx, video, ln1_w, ln1_b, W, b, ln2_w, ln2_b, PT, P, is_hu, offs):
        pd = W.shape[1]
        kp = (pd + 63) // 64 * 64                                      # K padded to the 64-deep GEMM step
        split = precise_split()
        f16 = vit_f16() and not precise_f32() and not vit_fp8() and not split
        lean = f16 and not any(ctx.needs_input_grad)      # eval forward: no bf16 xhat (backward only)
        xhat_p = K.patch_ln(video, is_hu, PT, P, offs, ld=kp, want_f16=f16, want_x3=split,
                            want_bf16=not lean)                                             # [M, kp], 0 pads
        if f16 or split:
            xhat_p, xhat16 = xhat_p      # bf16 (the weight gradient's operand) and fp16 (pair) (the GEMM's)
        xhat = xhat_p[:, :pd] if xhat_p is not None else None
        if split:
            # split-fp16 tower: the LayerNorm(4000) affine folded into the Linear in f32 (W diag(g),
            # b + W beta), then the x3 GEMM on the LayerNorm'd patches' fp16 pair
            bp = K.slinear(ln1_b.view(1, -1), W, bias=b).view(-1)
            y1, _ = K.linear_x3(xhat16, x3_weight(W, cols=kp, colscale=ln1_w, tag='patch'), bias=bp)
            del xhat16
        elif precise_f32():
            # f32 tower: LayerNorm(4000) with its affine, then the Linear, both exact f32
            # (ct_clip/ctvit.py:170-172); xhat (bf16) above is what the backward reads
            xn0 = K.patch_ln_f32(video, is_hu, PT, P, offs, ln1_w.detach(), ln1_b.detach())
            y1, _ = K.linear_f32(xn0, W.detach(), bias=b.detach())
            del xn0
        else:
            bp = K.slinear(ln1_b.view(1, -1), W, bias=b).view(-1)      # f32 [D]
            if f16:
                Wp = K.pack_rows_h16(W, W.shape[0], kp, colscale=ln1_w)   # fp16 [D, kp], zero pad columns
                y1 = K.linear(xhat16, Wp, bias=bp, out_dtype=F32)
                del xhat16
            else:
                Wp = K.pack_rows(W, W.shape[0], kp, colscale=ln1_w)    # bf16 [D, kp], zero pad columns
                y1 = K.linear(xhat_p, Wp, bias=bp, out_dtype=F32)       # [M, D]
        yb, yf, mean, rstd = K.layernorm_fwd(y1, ln2_w, ln2_b, 1e-5, out_bf16=True, out_f32=True)
        if lean:
            ctx.mark_non_differentiable(yb)
            return yf, yb
        ctx.save_for_backward(xhat, y1, mean, rstd, ln1_w, ln1_b, W, ln2_w)
        ctx.b, ctx.ln2_w, ctx.ln2_b = b, ln2_w, ln2_b
        ctx.mark_non_differentiable(yb)
        ctx.set_materialize_grads(False)   # no zero-filled grad for the bf16 companion
        return yf, yb

    @staticmethod
    def backward(ctx, dyf, _dyb):
        if dyf is None:   # the f32 output fed nothing that needs a gradient
            return (None,) * 11
        xhat, y1, mean, rstd, ln1_w, ln1_b, W, ln2_w = ctx.saved_tensors
        take_shadow(dyf)
        # LN2's gamma / beta gradients straight into their .grad (deferred partial reductions)
        _, dy1b, _, _ = K.layernorm_bwd(dyf.contiguous(), y1, mean, rstd, ln2_w, dx_f32=False,
                                        dgamma_out=gsink(ctx.ln2_w), dbeta_out=gsink(ctx.ln2_b))
        G = K.matmul_tn(dy1b, xhat, tag='dw')                           # [D, pd] f32
        cs = K.colsum(dy1b)                                             # d bias
        # straight into .grad (gsink), so the node's parameters are final when it returns
        # (dist_sync buckets fire on the node's post-hook, before any AccumulateGrad would run)
        sinks = [gsink(t) for t in (W, ln1_w, ln1_b)]
        tmp = [s_ if s_ is not None else torch.zeros_like(t) for s_, t in zip(sinks, (W, ln1_w, ln1_b))]
        K.patch_wgrad(G, cs, W, ln1_w, ln1_b, tmp[0], tmp[1], tmp[2], accumulate=True)
        if ctx.b.requires_grad:
            gsink(ctx.b).add_(cs)
        return None, None, None, None, None, None, None, None, None, None, None


# ----------------------------------------------------------------------------- reconstruction
class ReconFn(torch.autograd.Function):
    """``CTViT.to_pixels`` (ct_clip/ctvit.py:194-197: Linear(dim -> c*pt*p1*p2) + Rearrange to the
    video layout) and ``F.mse_loss(video, recon)`` (ctvit.py:451) as one node: the Linear is an MFMA
    GEMM with the bias epilogue, the rearrange + squared error + its gradient one HIP pass
    (``ctclip_unpatch_mse``) that never materialises the reconstruction unless it is returned.
    Returns (loss, recon or an empty tensor); the recon is not differentiable (the reference
    returns it detached from the loss as ``recon_video.clone()`` for logging)."""

    @staticmethod
    def forward(ctx, xf, xb, W, b, video, is_hu, PT, P, offs, want_recon):
        Wb = bf(W)
        pix = K.linear(xb, Wb, bias=b, out_dtype=F32)                   # [M, c*pt*p1*p2]
        loss, g, recon = K.unpatch_mse(pix, video, is_hu, PT, P, offs, want_grad=True, want_recon=want_recon)
        ctx.save_for_backward(xb, Wb, g)
        ctx.W, ctx.b = W, b
        if recon is None:
            recon = torch.empty(0, device=xf.device)
        ctx.mark_non_differentiable(recon)
        return loss.reshape(()), recon

    @staticmethod
    def backward(ctx, dloss, _drecon):
        xb, Wb, g = ctx.saved_tensors
        dpix = g * dloss                      # d loss / d pix, scaled by the incoming gradient
        dpb = K.cast_bf16(dpix)
        if ctx.W.requires_grad:
            K.matmul_tn(dpb, xb, out=gsink(ctx.W), accumulate=True)
        if ctx.b.requires_grad:
            K.colsum(dpix, out=gsink(ctx.b), accumulate=True)
        dx = K.matmul_nn(dpb, Wb, out_dtype=F32)
        return dx, None, None, None, None, None, None, None, None, None


# ----------------------------------------------------------------------------- CPB
def cpb_table(h, w, device):
    """Unique relative offsets of an h x w grid, log-spaced (ct_clip/attention.py:261-267):
    row bin = (dh + h-1)*(2w-1) + (dw + w-1)."""
    key = ('cpb', h, w, str(device))
    if key not in _MAP_CACHE:
        dh = torch.arange(-(h - 1), h).view(-1, 1).expand(2 * h - 1, 2 * w - 1)
        dw = torch.arange(-(w - 1), w).view(1, -1).expand(2 * h - 1, 2 * w - 1)
        rel = torch.stack([dh, dw], -1).reshape(-1, 2).to(torch.float32)
        rel = torch.sign(rel) * torch.log(rel.abs() + 1)
        _MAP_CACHE[key] = rel.contiguous().to(device)
    return _MAP_CACHE[key]


class CPBFn(torch.autograd.Function):
    """``ContinuousPositionBias`` (ct_clip/attention.py:229-276) evaluated on the 2,209 distinct
    offsets only (exact dedup of the 331,776 pairs).  Output u[heads][bin] (f32)."""

    @staticmethod
    def forward(ctx, rel, w0, b0, w1, b1, w2, b2):
        nb = rel.shape[0]
        H = w2.shape[0]
        h1 = K.slinear(rel, w0, b0, act=1)
        h2 = K.slinear(h1, w1, b1, act=1)
        u = torch.empty(H, nb, device=rel.device, dtype=F32)
        K.sgemm(nb, H, h2.shape[1], h2, h2.stride(0), 1, w2, 1, w2.stride(0), u, 1, nb, bias=b2)
        ctx.save_for_backward(rel, w0, w1, w2, h1, h2)
        ctx.params = (w0, b0, w1, b1, w2, b2)
        return u

    @staticmethod
    def backward(ctx, du):
        if getattr(ctx, '_ctclip_done', False):   # already run from the last layer's backward
            ctx._ctclip_done = False                 # (ctvit.encode_tokens: cpb_ready)
            return None, None, None, None, None, None, None
        rel, w0, w1, w2, h1, h2 = ctx.saved_tensors
        pw0, pb0, pw1, pb1, pw2, pb2 = ctx.params
        du = du.contiguous()
        H, nb = du.shape
        dev = du.device
        dz2 = torch.empty(nb, w2.shape[1], device=dev, dtype=F32)
        K.sgemm(nb, w2.shape[1], H, du, 1, nb, w2, w2.stride(0), 1, dz2, dz2.stride(0), 1, act=2, aux=h2,
                sxm=h2.stride(0), sxn=1)
        # parameter gradients accumulate straight into .grad
        if pw2.requires_grad:
            K.smm(du, h2, out=gsink(pw2), accumulate=True)
        if pb2.requires_grad:
            ones = torch.ones(nb, device=dev, dtype=F32)
            K.sgemm(H, 1, nb, du, nb, 1, ones, 1, 0, gsink(pb2), 1, 1, accumulate=True)
        if pw1.requires_grad:
            K.smm(dz2.t(), h1, out=gsink(pw1), accumulate=True)
        if pb1.requires_grad:
            K.colsum(dz2, out=gsink(pb1), accumulate=True)
        dz1 = K.smm(dz2, w1, act=2, aux=h1)
        if pw0.requires_grad:
            K.smm(dz1.t(), rel, out=gsink(pw0), accumulate=True)
        if pb0.requires_grad:
            K.colsum(dz1, out=gsink(pb0), accumulate=True)
        return None, None, None, None, None, None, None


# ----------------------------------------------------------------------------- transformer layer
def _bias_grad_ready(ctx, du):
    """The CPB table's gradient is complete once the first layer of the forward (the last backward)
    has run its attention backward: hand it to the owner's 'ready' callback right there (ctvit
    registers one that runs the CPB MLP's backward on the auxiliary stream), instead of when this
    layer's whole backward node returns."""
    if du is None or not ctx.bias_first:
        return
    cb = ctx.bias_acc.get('ready')
    if cb is not None:
        cb(du)


class ViTLayerFn(torch.autograd.Function):
    """One CTViT transformer layer (ct_clip/attention.py:322-331):
    x = PEG(x) + x; x = Attention(x, bias) + x; x = FeedForward(x) + x."""

    @staticmethod
    def forward(ctx, xf, xb, bias_u, geo, peg_w, peg_b, norm_g, q_scale, k_scale, Wq, Wkv, Wo, ff_w, ff_b, W1,
                W2):
        # the layers sharing one CPB table accumulate its gradient in ONE buffer (the attention's
        # slab reduction adds into it) and only the first layer of the forward -- the last backward
        # -- hands it to autograd: no per-layer gradient tensors for autograd to add up on the CPB
        # node's (auxiliary) stream
        if bias_u is not None:
            acc = bias_u.__dict__.setdefault('_ctclip_bias_acc', {'n': 0, 'du': None})
            ctx.bias_acc, ctx.bias_first = acc, acc['n'] == 0
            acc['n'] += 1
        if precise_f32() or precise_split():
            return _vit_layer_forward_f32(ctx, xf, xb, bias_u, geo, peg_w, peg_b, norm_g, q_scale, k_scale, Wq,
                                          Wkv, Wo, ff_w, ff_b, W1, W2, split=precise_split())
        H, dh = geo.heads, geo.dim_head
        inner = H * dh
        Wq_b, Wkv_b, Wo_b = bf(Wq), bf(Wkv), bf(Wo)
        fp8 = vit_fp8()
        dim = xb.shape[1]
        # the merged q | k l2norm backward of the fold (kernels.l2norm_qk_bwd_fold) is built for
        # exactly 256 q columns, the statistics merge (ctclip_ln_stats_merge) for <= 16 64-channel
        # groups: other widths run the unfolded LayerNorm + projections
        fold = not fp8 and _fold_shape_ok(geo, dim, Wkv)
        # fp16 forward GEMMs (vit_f16): the folded Q | K | V projection, to_out, FF1
        f16 = vit_f16() and fold and _PEG_X32
        # eval forward (round 6; no input needs a gradient, e.g. zero-shot inference under no_grad, the
        # VisionFeatureExtractor): none of the tensors only the backward reads is written -- the bf16
        # copies of x1, x2, LN(x2), O, the raw q / k, the attention LSE and FF1's h (~1.3 GB per layer
        # at B = 8)
        lean = f16 and not fp8 and not any(ctx.needs_input_grad)
        if _PEG_X32:
            x1f, x1b, x1h, m1, r1 = K.peg_fwd_x32(xf.detach().contiguous(), geo.B, geo.T, geo.Hg, geo.Wg, peg_w,
                                                  peg_b, geo.mode, stats=fold, want_f16=f16, want_bf16=not lean)
        elif fold:
            x1f, x1b, m1, r1 = K.peg_fwd_stats(xb, xf, geo.B, geo.T, geo.Hg, geo.Wg, peg_w, peg_b, geo.mode)
        else:
            x1f, x1b = K.peg_fwd(xb, xf, geo.B, geo.T, geo.Hg, geo.Wg, peg_w, peg_b, geo.mode)
        if fold:
            xn = None
        else:
            xn, _, m1, r1 = K.layernorm_fwd(x1f, norm_g, None, 1e-5)
        if fold:
            Wp, cs, scales = qkv_fold_pack(Wq, norm_g, Wkv, Wkv_b, q_scale, k_scale)
            if f16:
                Wp16, cs16 = qkv_fold_pack_h16(Wq, norm_g, Wkv, q_scale, k_scale)
                qkv, qkn = K.linear_qkv_lnfold(x1h, Wp16, cs16, m1, r1, scales, inner, 2 * inner,
                                               c_col0=2 * inner if lean else 0)
                del x1h, Wp16
            else:
                qkv, qkn = K.linear_qkv_lnfold(x1b, Wp, cs, m1, r1, scales, inner, 2 * inner)
            q, kv = qkv[:, :inner], qkv[:, inner:]
            qn, kn = qkn[:, :inner], qkn[:, inner:]
        elif fp8:
            q = fp8_linear(xn, Wq, 'q', Wq_b)
            kv = fp8_linear(x1b, Wkv, 'kv', Wkv_b)
            qn = K.l2norm_scale_fwd(q, H, dh, q_scale)
            kn = K.l2norm_scale_fwd(kv[:, :inner], H, dh, k_scale)
        elif _L2N_FUSED and dh == 32 and inner % 64 == 0:
            # l2norm(q) * q_scale, l2norm(k) * k_scale fused into the projections' epilogues (act 5)
            qn = torch.empty(xf.shape[0], inner, device=xf.device, dtype=BF16)
            kn = torch.empty(xf.shape[0], inner, device=xf.device, dtype=BF16)
            q = K.linear(xn, Wq_b, out2=qn, l2n_scale=q_scale.detach(), l2n_cols=inner)
            kv = K.linear(x1b, Wkv_b, out2=kn, l2n_scale=k_scale.detach(), l2n_cols=inner)
        else:
            q = K.linear(xn, Wq_b)
            kv = K.linear(x1b, Wkv_b)
            qn = K.l2norm_scale_fwd(q, H, dh, q_scale)
            kn = K.l2norm_scale_fwd(kv[:, :inner], H, dh, k_scale)
        L, nseq, seq = geo.seq()
        use_bias = bias_u is not None
        streams.mark_image_head(xf.device, 'attn')   # deferred text-stream work may start (streams.py)
        att = K.attn_fwd(qn, kn, kv[:, inner:], L=L, H=H, D=dh, nseq=nseq, scale=8.0, seq=seq,
                         bias_u=bias_u if use_bias else None, grid=(geo.Hg, geo.Wg) if use_bias else (0, 0),
                         want_o16=f16, eval_only=lean)
        o, lse = att[0], att[1]
        o_in, Wo_in = (att[2], h16(Wo)) if f16 else (o, Wo_b)   # to_out's operands
        # to_out + residual + the FeedForward's LayerNorm in one launch (gemm256.hip, EP -6) -- only
        # where a caller checks the launch's status word every step (kernels.ln_guard: the trainer)
        fused = None if fp8 or not K.ln_guarded() else K.linear_residual_ln(o_in, Wo_in, x1f, ff_w, ff_b, 1e-5,
                                                                            y16=f16, eval_only=lean)
        xn2h = None
        if fused is not None:
            x2f, x2b, xn2, m2, r2 = fused[:5]
            if f16:
                xn2h = fused[5]
        else:
            x2b = None if lean else torch.empty_like(xb)
            if fp8:
                x2f = fp8_linear(o, Wo, 'o', Wo_b, residual=x1f, out_f32=True, out2=x2b)
            else:
                x2f = K.linear(o_in, Wo_in, residual=x1f, out_dtype=F32, out2=x2b)
            lnr = K.layernorm_fwd(x2f, ff_w, ff_b, 1e-5, out_f16=f16, out_bf16=not lean)
            xn2, _, m2, r2 = lnr[:4]
            if f16:
                xn2h = lnr[4]
        del o_in, Wo_in
        W1p, W2p = pack_ff1(W1), pack_ff2(W2)
        g = torch.empty(xf.shape[0], W2p.shape[1], device=xf.device, dtype=BF16)
        x3b = torch.empty_like(xb)
        if fp8:
            h = fp8_linear(xn2, W1, 'ff1', W1p, act=K.ACT_GEGLU, out2=g)
            x3f = fp8_linear(g, W2, 'ff2', W2p, residual=x2f, out_f32=True, out2=x3b)
        elif f16:
            # fp16 FF1: h stored in fp16 (read by the GEGLU backward), g (bf16) from the fp16 h
            h = K.linear(xn2h, pack_ff1_h16(W1), act=K.ACT_GEGLU, out2=g, out_dtype=K.F16, tag='ff1',
                         flops=2.0 * xf.shape[0] * W1.shape[0] * W1.shape[1], discard_out=lean)
            del xn2h
            x3f = K.linear(g, W2p, residual=x2f, out_dtype=F32, out2=x3b)
        else:
            # tagged for bench.py's live roofline: algorithmic flops exclude the zero padding rows
            h = K.linear(xn2, W1p, act=K.ACT_GEGLU, out2=g, tag='ff1',
                         flops=2.0 * xf.shape[0] * W1.shape[0] * W1.shape[1])
            x3f = K.linear(g, W2p, residual=x2f, out_dtype=F32, out2=x3b)
        if lean:
            ctx.mark_non_differentiable(x3b)
            return x3f, x3b
        ctx.geo = geo
        ctx.use_bias = use_bias
        ctx.fold = fold
        ctx.fold_w = (Wp, cs) if fold else None
        ctx.params = (peg_w, peg_b, norm_g, q_scale, k_scale, Wq, Wkv, Wo, ff_w, ff_b, W1, W2)
        ctx.save_for_backward(xb, x1b, m1, r1, xn, q, kv, qn, kn, o, lse, x2b, m2, r2, xn2, h, g,
                              bias_u if use_bias else torch.empty(0), Wq_b, Wkv_b, Wo_b, W1p, W2p)
        ctx.mark_non_differentiable(x3b)
        ctx.set_materialize_grads(False)   # no zero-filled grad for the bf16 companion
        return x3f, x3b

    @staticmethod
    def backward(ctx, dx3f, _dx3b):
        if dx3f is None:   # the f32 output fed nothing that needs a gradient
            return (None,) * 16
        (xb, x1b, m1, r1, xn, q, kv, qn, kn, o, lse, x2b, m2, r2, xn2, h, g, bias_u, Wq_b, Wkv_b, Wo_b, W1p,
         W2p) = ctx.saved_tensors
        peg_w, peg_b, norm_g, q_scale, k_scale, Wq, Wkv, Wo, ff_w, ff_b, W1, W2 = ctx.params
        geo = ctx.geo
        H, dh = geo.heads, geo.dim_head
        inner = H * dh
        dev = dx3f.device
        dx3b = take_shadow(dx3f)          # bf16 image written by the next layer's PEG backward
        dx3f = dx3f.contiguous()
        if dx3b is None:
            dx3b = K.cast_bf16(dx3f)
        # feed-forward (weight gradients accumulate straight into the parameters' .grad)
        dh_ = K.matmul_nn_geglu_bwd(dx3b, W2p, h)      # dg = dx3 . W2 and the GEGLU backward, fused
        M_ = dx3b.shape[0]
        # weight gradients reduced from their split-K slabs straight into the unpacked .grad rows
        # (ctclip_reduce_slabs_rows: one pass instead of a slab reduction + unpack_rows)
        if gsink(W2) is not None:
            if _DW_UNPACK_FUSED:
                K.matmul_tn(dx3b, g, tag='dw', flops=2.0 * M_ * W2.shape[0] * W2.shape[1],
                            unpack=(gsink(W2), None, W2.shape[1]))
            else:
                K.unpack_rows(K.matmul_tn(dx3b, g, tag='dw', flops=2.0 * M_ * W2.shape[0] * W2.shape[1]), gsink(W2),
                              cols=W2.shape[1], accumulate=True)
        # dx2 = LN'(dh . W1) + dx3 in one launch where the shape allows (gemm256.hip, EP -7)
        fused = K.matmul_nn_ln_bwd(dh_, W1p, x2b, m2, r2, ff_w, dx3f, dgamma_out=gsink(ff_w),
                                   dbeta_out=gsink(ff_b)) if K.ln_guarded() else None
        if fused is None:
            if _DXN2_BLAS:    # A/B: hipBLASLt (torch.matmul) for this plain bf16 GEMM, W1 packed K-contiguous
                dxn2 = torch.matmul(dh_, W1p.t().contiguous().t())
            else:
                dxn2 = K.matmul_nn(dh_, W1p)
        if gsink(W1) is not None:
            rmap = ff1_rowmap(W1.shape[0] // 2, dev)
            if _DW_UNPACK_FUSED:
                K.matmul_tn(dh_, xn2, tag='dw', flops=2.0 * M_ * W1.shape[0] * W1.shape[1],
                            unpack=(gsink(W1), rmap, W1.shape[1]))
            else:
                K.unpack_rows(K.matmul_tn(dh_, xn2, tag='dw', flops=2.0 * M_ * W1.shape[0] * W1.shape[1]), gsink(W1),
                              rowmap=rmap, accumulate=True)
        if fused is not None:
            dx2f, dx2b = fused
        else:
            dx2f, dx2b, _, _ = K.layernorm_bwd(dxn2, x2b, m2, r2, ff_w, dres=dx3f, dgamma_out=gsink(ff_w),
                                               dbeta_out=gsink(ff_b))
        # attention
        do = K.matmul_nn(dx2b, Wo_b)
        K.matmul_tn(dx2b, o, out=gsink(Wo), accumulate=True, tag='dw')
        dqn = torch.empty_like(qn)
        dkn = torch.empty_like(kn)
        L, nseq, seq = geo.seq()
        du = None
        if ctx.use_bias:
            acc = ctx.bias_acc
            if acc['du'] is None:
                acc['du'] = torch.zeros_like(bias_u)
            du = acc['du']
        fold = getattr(ctx, 'fold', False)
        if fold:
            # the folded LayerNorm (ctx.fold, forward above) backward through the Q | K | V
            # projections without the LayerNorm output or its backward kernel:
            #   dqkv = [dq o rstd | dk | dv] (one buffer: the Q | K | V weight gradients are ONE GEMM)
            #   dWq = gamma o ((dq o rstd)^T x - u), dgamma = sum_n Wq o (...), dWkv = dkv^T x
            #   dx1 = LN'(dq Wq) + dkv Wkv + dx2 = dqkv [gamma o Wq ; Wkv] + dx2 - c1 - beta o x
            Wp, cs = ctx.fold_w
            M_ = qn.shape[0]
            dqkv = torch.empty(M_, 3 * inner, device=dev, dtype=BF16)
            dqkn = torch.empty(M_, 2 * inner, device=dev, dtype=BF16)       # [dq_n | dk_n]
            K.attn_bwd(qn, kn, kv[:, inner:], o, lse, do, dqkn[:, :inner], dqkn[:, inner:], dqkv[:, 2 * inner:],
                       L=L, H=H, D=dh, nseq=nseq, scale=8.0, seq=seq, bias_u=bias_u if ctx.use_bias else None,
                       dbias_u=du, grid=(geo.Hg, geo.Wg) if ctx.use_bias else (0, 0))
            _bias_grad_ready(ctx, du)
            if _QK_BWD_MERGED:
                # both l2norm backwards in one pass over the forward's [q | k] (one wave per row)
                qk = q.as_strided((M_, 2 * inner), q.stride())
                _, _, u1, c1, be1 = K.l2norm_qk_bwd_fold(qk, dqkn, q_scale, k_scale, r1, m1, dqkv[:, :2 * inner], cs,
                                                         x1b.shape[1], ds_q_out=gsink(q_scale),
                                                         ds_k_out=gsink(k_scale))
            else:
                _, _, u1, c1, be1 = K.l2norm_scale_bwd_fold(q, dqkn[:, :inner], H, dh, q_scale, r1, m1,
                                                            dx2=dqkv[:, :inner], fold_cs=cs, Dm=x1b.shape[1],
                                                            ds_out=gsink(q_scale))
                K.l2norm_scale_bwd(kv[:, :inner], dqkn[:, inner:], H, dh, k_scale, dqkv[:, inner:2 * inner],
                                   ds_out=gsink(k_scale))
            Gqkv = K.matmul_tn(dqkv, x1b, tag='dw')
            gq, gkv = gsink(Wq), gsink(Wkv)      # (frozen projections: scratch sinks)
            K.lnfold_wgrad(Gqkv, u1, norm_g, gq if gq is not None else torch.empty(Wq.shape, device=dev),
                           wq=Wq.detach(), grad_gamma=gsink(norm_g),
                           grad_rest=gkv if gkv is not None else torch.empty(Wkv.shape, device=dev))
            dx1f, dx1b = K.matmul_lnfold_bwd(dqkv, Wp, dx2f, x1b, c1, be1)
        else:
            dkv = torch.empty_like(kv)
            K.attn_bwd(qn, kn, kv[:, inner:], o, lse, do, dqn, dkn, dkv[:, inner:], L=L, H=H, D=dh, nseq=nseq,
                       scale=8.0, seq=seq, bias_u=bias_u if ctx.use_bias else None, dbias_u=du,
                       grid=(geo.Hg, geo.Wg) if ctx.use_bias else (0, 0))
            _bias_grad_ready(ctx, du)
            dq = torch.empty(q.shape, device=dev, dtype=q.dtype)
            K.l2norm_scale_bwd(q, dqn, H, dh, q_scale, dq, ds_out=gsink(q_scale))
            K.l2norm_scale_bwd(kv[:, :inner], dkn, H, dh, k_scale, dkv[:, :inner], ds_out=gsink(k_scale))
            fusable = K.ln_guarded() and K.ln_fusable(dq.shape[0], Wq_b.shape[1], bwd=True)
            if not fusable:
                dxn = K.matmul_nn(dq, Wq_b)
            K.matmul_tn(dq, xn, out=gsink(Wq), accumulate=True, tag='dw')
            K.matmul_tn(dkv, x1b, out=gsink(Wkv), accumulate=True, tag='dw')
            dx1kv = K.matmul_nn(dkv, Wkv_b, residual=dx2f, out_dtype=F32)
            # dx1 = LN'(dq . Wq) + (dkv . Wkv + dx2) in one launch where the shape allows (EP -7)
            fused = K.matmul_nn_ln_bwd(dq, Wq_b, x1b, m1, r1, norm_g, dx1kv, dgamma_out=gsink(norm_g)) \
                if fusable else None
            if fused is not None:
                dx1f, dx1b = fused
            else:
                if fusable:
                    dxn = K.matmul_nn(dq, Wq_b)
                dx1f, dx1b, _, _ = K.layernorm_bwd(dxn, x1b, m1, r1, norm_g, dres=dx1kv, want_beta=False,
                                                   dgamma_out=gsink(norm_g))
        # PEG
        # the weight / bias gradients accumulate into .grad in the slab-reduction launch itself, so the
        # layer's grads are final when its node returns (dist_sync buckets)
        dxf, dxb, _, _ = K.peg_bwd(dx1b, dx1f, xb, geo.B, geo.T, geo.Hg, geo.Wg, peg_w, geo.mode,
                                   dweight_out=gsink(peg_w), dbias_out=gsink(peg_b))
        put_shadow(dxf, dxb)
        if du is not None:
            if ctx.bias_first:       # every layer's share is in: release the buffer to autograd
                ctx.bias_acc['du'] = None
            else:
                du = None
        return (dxf, None, du, None, None, None, None, None, None, None, None, None, None,
                None, None, None)


def _fold_shape_ok(geo, dim, Wkv):
    """The LN1-folded Q | K | V path's shape conditions: the merged q | k l2norm backward of the fold
    (kernels.l2norm_qk_bwd_fold) is built for exactly 256 q columns, the statistics merge
    (ctclip_ln_stats_merge) for <= 16 64-channel groups."""
    inner = geo.heads * geo.dim_head
    return (_LN1_FOLD and _L2N_FUSED and geo.dim_head == 32 and inner == 256 and dim % 64 == 0 and dim <= 1024
            and geo.Wg <= 24 and Wkv.shape[0] == 2 * inner)


def _vit_layer_forward_f32(ctx, xf, xb, bias_u, geo, peg_w, peg_b, norm_g, q_scale, k_scale, Wq, Wkv, Wo, ff_w,
                           ff_b, W1, W2, split=False):
    """ViTLayerFn.forward of the f32 image tower: the layer (ct_clip/attention.py:322-331) with f32
    activations and exact-f32 products (every Linear on the f32 MFMA GEMM, PEG / LayerNorm / l2norm /
    cosine attention with the CPB bias / GEGLU in f32 with libm transcendentals), saving exactly the
    tensors ViTLayerFn.backward reads, as the bf16 forward saves them (bf16 copies of the f32
    activations; the attention's o / lse from the bf16 attention kernel on the bf16 q / k / v, so the
    backward's recomputed probabilities are those of its own operands).
    split (precise 'split' mode, round 6): the Linears on the x3 GEMM instead -- each operand an fp16
    (hi, lo) pair written by its producer (the f32-tap PEG, the LayerNorms, the x3 GEGLU epilogue; the
    attention output through ctclip_split_f16), ~22-bit operands with f32 accumulation -- and the PEG
    on the f32-tap x32 kernel; FF1's h is saved in fp16 (the GEGLU backward reads it as in the fp16
    default), g in bf16."""
    H, dh = geo.heads, geo.dim_head
    inner = H * dh
    d = lambda t: t.detach()    # noqa: E731
    # round 6: the backward is the default's LN1-folded one where the shape allows (ctx.fold; it reads
    # the LayerNorm statistics, x1 and the raw q | k | v in one bf16 [M, 3 inner] buffer, not the
    # LayerNorm output): the Q-side LayerNorm writes no bf16 copy and the backward runs no LayerNorm
    # backward kernel -- the same backward kernels as the default tower
    fold = _fold_shape_ok(geo, xf.shape[1], Wkv)
    qkvb = torch.empty(xf.shape[0], 3 * inner, device=xf.device, dtype=BF16) if fold else None
    qb_out = qkvb[:, :inner] if fold else None
    kvb_out = qkvb[:, inner:] if fold else None
    if split:
        x1f, x1b, x1s, _, _ = K.peg_fwd_x32(xf.detach().contiguous(), geo.B, geo.T, geo.Hg, geo.Wg, d(peg_w),
                                            d(peg_b), geo.mode, want_x3=True)
        xn, _, m1, r1, xns = K.layernorm_fwd(x1f, norm_g, None, 1e-5, out_bf16=not fold, out_x3=True)  # q side
        q32, q = K.linear_x3(xns, x3_weight(Wq), want_bf16=True, out_bf16=qb_out)
        kv32, kv = K.linear_x3(x1s, x3_weight(Wkv), want_bf16=True, out_bf16=kvb_out)   # K / V: un-normalised x
        del xns, x1s
    else:
        x1f = K.peg_fwd_f32(xf.detach().contiguous(), geo.B, geo.T, geo.Hg, geo.Wg, d(peg_w), d(peg_b), geo.mode)
        x1b = K.cast_bf16(x1f)
        xn, xnf, m1, r1 = K.layernorm_fwd(x1f, norm_g, None, 1e-5, out_bf16=not fold, out_f32=True)   # q side
        q32, q = K.linear_f32(xnf, d(Wq), want_bf16=True, out_bf16=qb_out)
        kv32, kv = K.linear_f32(x1f, d(Wkv), want_bf16=True, out_bf16=kvb_out)   # K / V from the un-normalised x
        del xnf
    ctx.fold = fold
    ctx.fold_w = qkv_fold_pack(Wq, norm_g, Wkv, bf(Wkv), q_scale, k_scale)[:2] if fold else None
    return _vit_layer_tail_f32(ctx, x1f, x1b, xn, m1, r1, q32, q, kv32, kv, xb, bias_u, geo, peg_w, peg_b, norm_g,
                               q_scale, k_scale, Wq, Wkv, Wo, ff_w, ff_b, W1, W2, split=split)


def _vit_layer_tail_f32(ctx, x1f, x1b, xn, m1, r1, q32, q, kv32, kv, xb, bias_u, geo, peg_w, peg_b, norm_g, q_scale,
                        k_scale, Wq, Wkv, Wo, ff_w, ff_b, W1, W2, split):
    """_vit_layer_forward_f32 from the f32 q / kv on: l2norm, attention, to_out, FeedForward."""
    H, dh = geo.heads, geo.dim_head
    inner = H * dh
    d = lambda t: t.detach()    # noqa: E731
    # the l2norms write the bf16 copies the backward reads (and the bf16 attention below) themselves
    qn = torch.empty(q32.shape[0], inner, device=q32.device, dtype=BF16)
    kn = torch.empty(q32.shape[0], inner, device=q32.device, dtype=BF16)
    qn32 = K.l2norm_scale_fwd_f32(q32, H, dh, d(q_scale), out_bf16=qn)
    kn32 = K.l2norm_scale_fwd_f32(kv32[:, :inner], H, dh, d(k_scale), out_bf16=kn)
    L, nseq, seq = geo.seq()
    use_bias = bias_u is not None
    grid = (geo.Hg, geo.Wg) if use_bias else (0, 0)
    if split and dh == 32:
        # x3 attention: O straight as to_out's fp16 pair, plus the bf16 O / LSE the backward reads
        os_, o, lse = K.attn_fwd_x3(qn32, kn32, kv32[:, inner:], L=L, H=H, D=dh, nseq=nseq, scale=8.0, seq=seq,
                                    bias_u=bias_u if use_bias else None, grid=grid)
        del q32, qn32, kn32
        o32 = None
    else:
        o32 = K.attn_fwd_f32(qn32, kn32, kv32[:, inner:], L=L, H=H, D=dh, nseq=nseq, scale=8.0, seq=seq,
                             bias_u=bias_u if use_bias else None, grid=grid)
        del q32, qn32, kn32
        o, lse = K.attn_fwd(qn, kn, kv[:, inner:], L=L, H=H, D=dh, nseq=nseq, scale=8.0, seq=seq,
                            bias_u=bias_u if use_bias else None, grid=grid)
        os_ = K.split_f16(o32) if split else None
    inner_ff = W1.shape[0] // 2
    if split:
        x2f, x2b = K.linear_x3(os_, x3_weight(Wo), residual=x1f, want_bf16=True)
        del o32, os_, kv32, x1f
        xn2, _, m2, r2, xn2s = K.layernorm_fwd(x2f, ff_w, ff_b, 1e-5, out_bf16=True, out_x3=True)
        W1s = x3_weight(W1, rows=2 * ff_pad(inner_ff), rowmap=ff1_rowmap(inner_ff, W1.device), tag='ff1')
        h, gs, g = K.linear_x3_geglu(xn2s, W1s, tag='ff1', flops=2.0 * x2f.shape[0] * W1.shape[0] * W1.shape[1])
        del xn2s
        x3f, x3b = K.linear_x3(gs, x3_weight(W2, cols=ff_pad(W2.shape[1]), tag='ff2'), residual=x2f, want_bf16=True)
        del gs
    else:
        x2f, x2b = K.linear_f32(o32, d(Wo), residual=x1f, want_bf16=True)
        del o32, kv32, x1f
        xn2, xn2f, m2, r2 = K.layernorm_fwd(x2f, ff_w, ff_b, 1e-5, out_bf16=True, out_f32=True)
        W1p32 = K.pack_rows_f32(d(W1), 2 * ff_pad(inner_ff), W1.shape[1], rowmap=ff1_rowmap(inner_ff, W1.device))
        h, g32, g = K.linear_f32_geglu(xn2f, W1p32)
        del xn2f
        W2p32 = K.pack_rows_f32(d(W2), W2.shape[0], ff_pad(W2.shape[1]))
        x3f, x3b = K.linear_f32(g32, W2p32, residual=x2f, want_bf16=True)
        del g32
    ctx.geo = geo
    ctx.use_bias = use_bias
    ctx.params = (peg_w, peg_b, norm_g, q_scale, k_scale, Wq, Wkv, Wo, ff_w, ff_b, W1, W2)
    # (ctx.fold / fold_w set by _vit_layer_forward_f32; with the fold xn is None)
    ctx.save_for_backward(xb, x1b, m1, r1, xn, q, kv, qn, kn, o, lse, x2b, m2, r2, xn2, h, g,
                          bias_u if use_bias else torch.empty(0), bf(Wq), bf(Wkv), bf(Wo), pack_ff1(W1), pack_ff2(W2))
    ctx.mark_non_differentiable(x3b)
    ctx.set_materialize_grads(False)   # no zero-filled grad for the bf16 companion
    return x3f, x3b


class NormFn(torch.autograd.Function):
    """Bias-less LayerNorm ``norm_out`` (ct_clip/attention.py:309,333) -> (f32, bf16)."""

    @staticmethod
    def forward(ctx, xf, xb, gamma):
        yb, yf, mean, rstd = K.layernorm_fwd(xf, gamma, None, 1e-5, out_bf16=True, out_f32=True)
        ctx.save_for_backward(xb, mean, rstd, gamma)
        ctx.gamma = gamma
        ctx.mark_non_differentiable(yb)
        ctx.set_materialize_grads(False)   # no zero-filled grad for the bf16 companion
        return yf, yb

    @staticmethod
    def backward(ctx, dyf, _):
        if dyf is None:   # the f32 output fed nothing that needs a gradient
            return None, None, None
        xb, mean, rstd, gamma = ctx.saved_tensors
        take_shadow(dyf)
        dxf, dxb, _, _ = K.layernorm_bwd(dyf.contiguous(), xb, mean, rstd, gamma, want_beta=False,
                                         dgamma_out=gsink(ctx.gamma))
        put_shadow(dxf, dxb)
        return dxf, None, None


# ----------------------------------------------------------------------------- VQ + pooling
class VQPoolFn(torch.autograd.Function):
    """``vq`` (ct_clip/ctvit.py:421-427; vector_quantize_pytorch cosine codebook) followed by the
    pooling of CTCLIP.forward (ct_clip.py:724,740): mean over t, flatten (h, w, d).
    Straight-through estimator in training; codebook EMA update in training mode (buffers
    updated in place AFTER the quantised values are read, as the reference does; all-reduced
    across ranks so every rank keeps the same codebook).  Optionally also returns the full
    quantised token tensor codebook[idx] ([M, D] f32)."""

    @staticmethod
    def forward(ctx, zf, zb, embed, cluster, geo, training, decay, state, want_tokens):
        ctx.set_materialize_grads(False)
        D = zf.shape[1]
        C = embed.shape[-2]
        cb = embed.view(C, D)
        state.flush_ema()               # a previous call's deferred EMA update, queued before ...
        streams.join_aux(zf.device)     # ... this wait for the previous step's codebook update
        idx, xn = vq_assign(zf, zb, cb, state, want_xn=training)
        cb_b = state.codebook_bf16(cb)   # the mirror vq_assign scored against (cached)
        HW = geo.Hg * geo.Wg
        pooled, pooled_b = K.vq_pool(idx, cb, geo.B, geo.T, HW)
        tokens = K.vq_gather(idx, cb) if want_tokens else torch.empty(0, device=zf.device)
        if training:
            # EMA update on the auxiliary stream (streams.py): after the pool / gather above have
            # read the pre-update codebook, beside the rest of this step
            aux = streams.aux_stream(zf.device)

            def ema():
                # persistent statistics (2^-40 fixed-point esum), zeroed once here and then by the
                # finalize kernel behind its reads: no fill launches per step.  bins has one slot past
                # the C counts: this rank's step status word (a flagged forward: fp16 range, a
                # non-finite token, a LayerNorm exchange timeout), summed over the ranks with the
                # statistics, so every rank drops a flagged step's codebook update together
                bins_g, esum = state.ema_buffers(C, D, zf.device)
                bins = bins_g[:C]
                if zf.is_cuda:
                    # the guard: the trainer's summed skip word of this update's step when it owns the
                    # step (DEFER_EMA '2' / '3': the update may run beside the NEXT step, whose
                    # kernels may flag the live word for their own step), else the live word
                    g_src, state.ema_guard = state.ema_guard, None
                    bins_g[C:].copy_(g_src if g_src is not None else K.status_word(zf.device))
                work = state.ema_work(C, xn.shape[0], zf.device) if _EMA_SORTED else None
                K.vq_ema_accum(idx, xn, bins, esum, work=work)
                dist_sync.sum_codebook_stats(bins_g, esum)
                K.vq_ema_finalize(bins, esum, decay, cb, cluster.view(-1), cb_b, reset=True,
                                  guard=bins_g[C:] if zf.is_cuda else None)
            if aux is None:
                ema()
            else:
                dev = zf.device

                def launch():
                    aux.wait_stream(torch.cuda.current_stream(dev))
                    for t in (idx, xn, cb, cluster, cb_b):
                        t.record_stream(aux)
                    with torch.cuda.stream(aux):
                        ema()
                # CTCLIP.encode defers the launch until after the image projection: the EMA's
                # statistics pass (~0.36 ms, HBM-bound) otherwise runs beside the projection's
                # weight stream (302 MB) and slows it by ~40 us (r05f: 98 us in step vs 56 alone)
                if state.defer_ema:
                    state.pending_ema = launch
                else:
                    launch()
            state.mark_codebook_fresh(cb)
        ctx.geo = geo
        ctx.D = D
        state.last_indices = idx
        ctx.mark_non_differentiable(pooled_b)
        return pooled, pooled_b, tokens

    @staticmethod
    def backward(ctx, dpooled, _, dtokens):
        geo = ctx.geo
        dz = None
        if dpooled is not None:
            dz, _ = K.vq_pool_bwd(dpooled.contiguous(), geo.B, geo.T, geo.Hg * geo.Wg, ctx.D)
        if dtokens is not None and dtokens.numel():
            dz = dtokens.contiguous() if dz is None else dz + dtokens
        return dz, None, None, None, None, None, None, None, None


# the VQ distance GEMM on fp16 operands (round 6; CTCLIP_VQ_F16=0: bf16): l2norm(zf) and the codebook
# each rounded once at 2^-11, so the f32 re-score margin is 4e-3 instead of 2e-2 and vq_select
# re-scores ~3x fewer codes; same exact f32 argmax
_VQ_F16 = os.environ.get('CTCLIP_VQ_F16', '1') != '0'


def vq_assign(zf, zb, cb, state, want_xn=False):
    """Cosine-codebook assignment (vector_quantize_pytorch cosine sim + argmax, ct_clip/ctvit.py:427):
    16-bit MFMA distance GEMM with a per-64-code-group (best, index, second-best) epilogue -- fp16
    l2norm(zf) against the fp16 codebook image (bf16 l2norm(zb) and codebook with CTCLIP_VQ_F16=0)
    -- then the f32 re-score of every code within that GEMM's error margin (vq.hip) -> the exact
    f32 argmax of l2norm(zf) . cb^T.  Returns (idx int32 [M], l2norm(zf) f32 or None)."""
    D = zf.shape[1]
    C = cb.shape[0]
    if _VQ_F16 and D % 64 == 0:
        xn_s = K.vq_l2norm_h16(zf)
        cb_s = K.split_f16(cb)[0]       # (the EMA updates cb in place: cast per call, 4 M elements)
        margin = 4e-3
    else:
        xn_s = K.l2norm_scale_fwd(zb, 1, D, state.ones(D, zf.device))
        cb_s = state.codebook_bf16(cb)
        margin = 2e-2
    nt = (C + 63) // 64
    cand = torch.empty(zf.shape[0], nt, 2, device=zf.device, dtype=F32)
    cand2 = torch.empty(zf.shape[0], nt, device=zf.device, dtype=F32)
    K.gemm_raw(zf.shape[0], C, D, xn_s, D, True, cb_s, D, True, cand, nt, C2=cand2, ldc2=nt, act=K.ACT_ARGMAX)
    return K.vq_select(cand, zf, cb, margin=margin, want_xn=want_xn, cand2=cand2)


class VQState:
    """Caches of the vector quantiser: bf16 codebook mirror and constant vectors."""

    def __init__(self):
        self._cb = None
        self._cb_ver = None
        self._ones = {}
        self.last_indices = None
        self.defer_ema = False      # VQPoolFn leaves its EMA launch in pending_ema (CTCLIP.encode)
        self.pending_ema = None
        self.ema_guard = None       # int32[1] guard word for the pending update (CTClipTrainer)

    def ema_buffers(self, C, D, device):
        """(bins f32 [C + 1], esum int64 [C, D]) of the EMA update, zero between updates (created on the
        stream of the first update, which every later update also runs on); bins[C] is the guard slot
        (the step status word, VQPoolFn.forward)."""
        b = getattr(self, '_ema_buf', None)
        if b is None or b[1].shape != (C, D) or b[1].device != device:
            b = (torch.zeros(C + 1, device=device, dtype=F32), torch.zeros(C, D, device=device, dtype=torch.int64))
            self._ema_buf = b
        return b

    def ema_work(self, C, rows, device):
        """int32 scratch of the code-sorted EMA accumulation (kernels.vq_ema_accum): 2 C + 2 rows
        entries, the first C zero between updates (the kernels leave them zero); grown as needed."""
        w = getattr(self, '_ema_work', None)
        n = 2 * C + 2 * rows
        if w is None or w.numel() < n or w.device != device:
            w = torch.zeros(n, device=device, dtype=torch.int32)
            self._ema_work = w
        return w

    def flush_ema(self):
        """Queue a deferred codebook EMA update (on the auxiliary stream, after the current stream's
        work so far).  Every reader of the codebook calls this first."""
        fn, self.pending_ema = self.pending_ema, None
        if fn is not None:
            fn()

    def codebook_bf16(self, cb):
        key = (cb.data_ptr(), cb._version)
        if self._cb is None or self._cb_ver != key:
            self._cb = K.cast_bf16(cb)
            self._cb_ver = key
        return self._cb

    def mark_codebook_fresh(self, cb):
        self._cb_ver = (cb.data_ptr(), cb._version)

    def ones(self, D, device):
        k = (D, str(device))
        if k not in self._ones:
            self._ones[k] = torch.ones(D, device=device, dtype=F32)
        return self._ones[k]


# ----------------------------------------------------------------------------- projections
class ImageProjFn(torch.autograd.Function):
    """``to_visual_latent`` Linear(dim_image -> dim_latent, no bias) (ct_clip/ct_clip.py:564,767)
    as a split-K bf16 MFMA GEMM (the 294,912-wide weight is read once per step)."""

    @staticmethod
    def forward(ctx, pooled, pooled_b, W, Wb):
        ctx.save_for_backward(pooled_b, Wb)
        ctx.W = W
        if precise_f32() or precise_split():
            # the precise towers' projection in f32: the HBM-streaming skinny GEMM on the f32 weight
            # (ctclip_skinny_sgemm, an f32 fma per product; 604 MB read once), else split-K f32 MFMA
            out = K.skinny_linear(pooled.detach().contiguous(), W.detach()) if _SKINNY_PROJ else None
            return out if out is not None else K.slinear(pooled.detach().contiguous(), W.detach())
        # the HBM-streaming skinny GEMM (csrc/proj.hip): the 302 MB weight read once at ~HBM speed
        # (the generic split-K 128-row MFMA tile ran at 0.85 TB/s at M = 8, round 4)
        if _SKINNY_PROJ:
            out = K.skinny_linear(pooled_b, Wb)
            if out is not None:
                return out
        B, Kd = pooled_b.shape
        N = Wb.shape[0]
        split = max(1, min(512, Kd // 1024))
        slabs = torch.empty(split, B, N, device=pooled.device, dtype=F32)
        K.gemm_raw(B, N, Kd, pooled_b, Kd, True, Wb, Kd, True, slabs, N, split_k=split)
        out = torch.empty(B, N, device=pooled.device, dtype=F32)
        K.reduce_slabs(slabs, out)
        return out

    @staticmethod
    def backward(ctx, dout):
        pooled_b, Wb = ctx.saved_tensors
        dlb = K.cast_bf16(dout.contiguous())
        dpooled = K.matmul_nn(dlb, Wb, out_dtype=F32) if ctx.needs_input_grad[0] else None
        if ctx.needs_input_grad[2]:   # the 294,912-wide weight gradient lands in .grad directly
            K.matmul_tn(dlb, pooled_b, out=gsink(ctx.W), accumulate=True)
        return dpooled, None, None, None


class TextProjFn(torch.autograd.Function):
    """``to_text_latent`` Linear(768 -> 512, no bias) on the CLS row (ct_clip/ct_clip.py:549,762-765),
    exact f32."""

    @staticmethod
    def forward(ctx, cls, W):
        ctx.save_for_backward(cls, W)
        ctx.W = W
        return K.slinear(cls, W)

    @staticmethod
    def backward(ctx, dout):
        cls, W = ctx.saved_tensors
        dout = dout.contiguous()
        dcls = K.smm(dout, W) if ctx.needs_input_grad[0] else None
        if ctx.needs_input_grad[1]:
            K.smm(dout.t(), cls, out=gsink(ctx.W), accumulate=True)
        return dcls, None


# ----------------------------------------------------------------------------- loss

class ClipLossFn(torch.autograd.Function):
    """Symmetric InfoNCE (ct_clip/ct_clip.py:845-901).  Under torch.distributed the raw latents
    are all-gathered (RCCL) so the negatives span the global batch; every rank computes the
    same global loss and back-propagates its own rows (gradients are then SUM-reduced)."""

    @staticmethod
    def forward(ctx, t_raw, i_raw, log_temp, impl=None, t_gather=None):
        B = t_raw.shape[0]
        tg, ig = dist_sync.gather_latents(t_raw, i_raw, t_gather)
        # impl: the fused HIP loss (default); tests substitute a CPU restatement to exercise
        # the exchange logic under gloo
        loss, dt, di, dlt = (impl or K.clip_loss)(tg, ig, log_temp.reshape(1).contiguous())[:4]
        ctx.save_for_backward(dist_sync.local_rows(dt, B), dist_sync.local_rows(di, B), dlt)
        ctx.scale = dist_sync.replicated_grad_scale()
        return loss.reshape(())

    @staticmethod
    def backward(ctx, dloss):
        dt, di, dlt = ctx.saved_tensors
        s = dloss.reshape(1)
        # log-temperature gradient: every rank holds the full global value -> scaled by 1/world so
        # the SUM all-reduce reproduces it once.
        return dt * s, di * s, (dlt * s * ctx.scale).reshape(()), None, None


# ----------------------------------------------------------------------------- BERT
class BertEmbedFn(torch.autograd.Function):
    """BertEmbeddings: word + position + token_type(0), LayerNorm(eps 1e-12)."""

    @staticmethod
    def forward(ctx, ids, word, pos, typ, ln_w, ln_b, eps, drop=(0.0, 0), pad_id=-1):
        x = K.embed_fwd(ids, word, pos, typ[0])
        ctx.pad_id = pad_id
        if drop[0] > 0:
            _, yf, mean, rstd = K.layernorm_fwd(x, ln_w, ln_b, eps, out_bf16=False, out_f32=True)
            yf, yb = K.dropout(yf, drop[0], drop[1], out_f32=True, out_bf16=True)
        else:
            yb, yf, mean, rstd = K.layernorm_fwd(x, ln_w, ln_b, eps, out_bf16=True, out_f32=True)
        ctx.drop = drop
        ctx.save_for_backward(ids, x, mean, rstd, ln_w)
        ctx.params = (word, pos, typ, ln_w, ln_b)
        ctx.mark_non_differentiable(yb)
        ctx.set_materialize_grads(False)   # no zero-filled grad for the bf16 companion
        return yf, yb

    @staticmethod
    def backward(ctx, dyf, _):
        if dyf is None:   # the f32 output fed nothing that needs a gradient
            return (None,) * 9
        ids, x, mean, rstd, ln_w = ctx.saved_tensors
        word, pos, typ, _, ln_b = ctx.params
        dyf = dyf.contiguous()
        if ctx.drop[0] > 0:
            dyf = K.dropout(dyf, ctx.drop[0], ctx.drop[1])[0]
        dx, _, _, _ = K.layernorm_bwd(dyf, x, mean, rstd, ln_w, dx_bf16=False,
                                      dgamma_out=gsink(ln_w), dbeta_out=gsink(ln_b))
        dtyp = gsink(typ)
        # accumulated straight into the parameters' .grad; the pad id's row gets nothing
        # (padding_idx of transformers' BertEmbeddings word table)
        K.embed_bwd(ids, dx, gsink(word), gsink(pos), dtyp[0] if dtyp is not None else None, ctx.pad_id)
        return None, None, None, None, None, None, None, None, None


class BertLayerFn(torch.autograd.Function):
    """One BertLayer (post-LN): self-attention (fused QKV GEMM + MFMA attention, scale 1/sqrt(d),
    additive key mask) -> dense + residual -> LN -> GELU MLP -> dense + residual -> LN."""

    @staticmethod
    def forward(ctx, xf, xb, kmask, B, L, heads, eps, Wq, bq, Wk, bk, Wv, bv, Wo, bo, ln1_w, ln1_b, Wi, bi, Wout,
                bout, ln2_w, ln2_b, drop=(0.0, 0.0, 0, 0, 0), split=None):
        ph, pa, s_attn, s_out1, s_out2 = drop
        Hd = xf.shape[1]
        dh = Hd // heads
        split = _TEXT_SPLIT if split is None else (split and _TEXT_SPLIT)
        if split:
            (Wqkv, Wqkv_lo), (Wo_b, Wo_lo), (Wi_b, Wi_lo), (Wout_b, Wout_lo) = (
                bf_cat_split([Wq, Wk, Wv]), bf_split(Wo), bf_split(Wi), bf_split(Wout))
        else:
            Wqkv, Wo_b, Wi_b, Wout_b = bf_cat([Wq, Wk, Wv]), bf(Wo), bf(Wi), bf(Wout)
            Wqkv_lo = Wo_lo = Wi_lo = Wout_lo = None
        bqkv = cat_f32([bq, bk, bv])
        qkv = K.linear(xb, Wqkv, bias=bqkv, w_lo=Wqkv_lo)
        ctxv, lse = K.attn_fwd(qkv[:, :Hd], qkv[:, Hd:2 * Hd], qkv[:, 2 * Hd:], L=L, H=heads, D=dh, nseq=B,
                               scale=1.0 / math.sqrt(dh), seq=(1, L, 0, 1), kmask=kmask, dropout=(pa, s_attn))
        if ph > 0 and _BERT_FUSE:   # LN(dropout(dense(ctx)) + x): the dropout in the split-K combine
            a = K.linear(ctxv, Wo_b, bias=bo, residual=xf, out_dtype=F32, w_lo=Wo_lo, dropout=(ph, s_out1))
        elif ph > 0:     # (A/B: the stand-alone dropout kernel; the residual leaves the GEMM epilogue)
            a = K.dropout(K.linear(ctxv, Wo_b, bias=bo, out_dtype=F32, w_lo=Wo_lo), ph, s_out1, res=xf)[0]
        else:
            a = K.linear(ctxv, Wo_b, bias=bo, residual=xf, out_dtype=F32, w_lo=Wo_lo)
        x1b, x1f, m1, r1 = K.layernorm_fwd(a, ln1_w, ln1_b, eps, out_bf16=True, out_f32=True)
        hpre = torch.empty(xf.shape[0], Wi.shape[0], device=xf.device, dtype=BF16)
        hact = K.linear(x1b, Wi_b, bias=bi, act=K.ACT_GELU, out2=hpre, w_lo=Wi_lo)
        if ph > 0 and _BERT_FUSE:
            b2 = K.linear(hact, Wout_b, bias=bout, residual=x1f, out_dtype=F32, w_lo=Wout_lo, dropout=(ph, s_out2))
        elif ph > 0:
            b2 = K.dropout(K.linear(hact, Wout_b, bias=bout, out_dtype=F32, w_lo=Wout_lo), ph, s_out2, res=x1f)[0]
        else:
            b2 = K.linear(hact, Wout_b, bias=bout, residual=x1f, out_dtype=F32, w_lo=Wout_lo)
        x2b, x2f, m2, r2 = K.layernorm_fwd(b2, ln2_w, ln2_b, eps, out_bf16=True, out_f32=True)
        ctx.save_for_backward(xb, kmask, qkv, ctxv, lse, a, m1, r1, x1b, hpre, hact, b2, m2, r2, Wqkv, Wo_b, Wi_b,
                              Wout_b, ln1_w, ln2_w)
        ctx.params = (Wq, bq, Wk, bk, Wv, bv, Wo, bo, ln1_w, ln1_b, Wi, bi, Wout, bout, ln2_w, ln2_b)
        ctx.dims = (B, L, heads, dh)
        ctx.drop = drop
        ctx.mark_non_differentiable(x2b)
        ctx.set_materialize_grads(False)   # no zero-filled grad for the bf16 companion
        return x2f, x2b

    @staticmethod
    def backward(ctx, dx2f, _):
        if dx2f is None:   # the f32 output fed nothing that needs a gradient
            return (None,) * 25
        (xb, kmask, qkv, ctxv, lse, a, m1, r1, x1b, hpre, hact, b2, m2, r2, Wqkv, Wo_b, Wi_b, Wout_b, ln1_w,
         ln2_w) = ctx.saved_tensors
        Wq, bq, Wk, bk, Wv, bv, Wo, bo, _, ln1_b, Wi, bi, Wout, bout, _, ln2_b = ctx.params
        B, L, heads, dh = ctx.dims
        ph, pa, s_attn, s_out1, s_out2 = ctx.drop
        Hd = heads * dh

        def wgrad(dy, x, W, b, bias_done=False):   # dW += dy^T x, db += colsum(dy), into .grad
            if W.requires_grad:
                K.matmul_tn(dy, x, out=gsink(W), accumulate=True)
            if b.requires_grad and not bias_done:
                K.colsum(dy, out=gsink(b), accumulate=True)

        fuse = ph > 0 and _BERT_FUSE
        # LN2 + FF out; with dropout the LN backward also emits the dense branch's masked bf16
        # gradient and its column sums (the dense bias gradient)
        if fuse:
            db2f, db2b = K.layernorm_bwd_drop(dx2f.contiguous(), b2, m2, r2, ln2_w, ph, s_out2,
                                              dgamma_out=gsink(ln2_w), dbeta_out=gsink(ln2_b),
                                              dbias_out=gsink(bout) if bout.requires_grad else None)
        else:
            db2f, db2b, _, _ = K.layernorm_bwd(dx2f.contiguous(), b2, m2, r2, ln2_w, dgamma_out=gsink(ln2_w),
                                               dbeta_out=gsink(ln2_b))
            if ph > 0:       # gradient through the output dropout (the residual path bypasses it)
                db2b = K.dropout(db2f, ph, s_out2, out_f32=False, out_bf16=True)[1]
        if _BERT_FUSE:       # dhpre = (db2 . Wout) * gelu'(hpre) in one GEMM (act 6)
            dhpre = K.matmul_nn_gelu_bwd(db2b, Wout_b, hpre)
        else:
            dhpre = K.gelu_bwd(K.matmul_nn(db2b, Wout_b), hpre)
        wgrad(db2b, hact, Wout, bout, bias_done=fuse)
        dx1 = K.matmul_nn(dhpre, Wi_b, residual=db2f, out_dtype=F32)
        wgrad(dhpre, x1b, Wi, bi)
        # LN1 + attention out
        if fuse:
            daf, dab = K.layernorm_bwd_drop(dx1, a, m1, r1, ln1_w, ph, s_out1, dgamma_out=gsink(ln1_w),
                                            dbeta_out=gsink(ln1_b), dbias_out=gsink(bo) if bo.requires_grad else None)
        else:
            daf, dab, _, _ = K.layernorm_bwd(dx1, a, m1, r1, ln1_w, dgamma_out=gsink(ln1_w),
                                             dbeta_out=gsink(ln1_b))
            if ph > 0:
                dab = K.dropout(daf, ph, s_out1, out_f32=False, out_bf16=True)[1]
        dctx = K.matmul_nn(dab, Wo_b)
        wgrad(dab, ctxv, Wo, bo, bias_done=fuse)
        dqkv = torch.empty_like(qkv)
        K.attn_bwd(qkv[:, :Hd], qkv[:, Hd:2 * Hd], qkv[:, 2 * Hd:], ctxv, lse, dctx, dqkv[:, :Hd],
                   dqkv[:, Hd:2 * Hd], dqkv[:, 2 * Hd:], L=L, H=heads, D=dh, nseq=B, scale=1.0 / math.sqrt(dh),
                   seq=(1, L, 0, 1), kmask=kmask, dropout=(pa, s_attn))
        dx = K.matmul_nn(dqkv, Wqkv, residual=daf, out_dtype=F32)
        gW, gB = (gsink_cat([Wq, Wk, Wv]), gsink_cat([bq, bk, bv])) if _QKV_WGRAD else (None, None)
        if gW is not None and gB is not None:
            # q / k / v gradients adjacent in the arena: one [3 Hd, Hd] weight-gradient GEMM (108
            # tiles instead of 3 x 36) and one column sum, same per-element arithmetic
            K.matmul_tn(dqkv, xb, out=gW, accumulate=True)
            K.colsum(dqkv, out=gB, accumulate=True)
        else:
            for i, (W, b) in enumerate(((Wq, bq), (Wk, bk), (Wv, bv))):
                wgrad(dqkv[:, i * Hd:(i + 1) * Hd], xb, W, b)
        return (dx, None, None, None, None, None, None) + (None,) * 18
