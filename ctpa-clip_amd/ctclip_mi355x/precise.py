"""Opt-in f32 image tower: the 3D-ViT forward (and the image projection) with f32 activations and
exact-f32 products, for outputs that must match the reference's fp32 run index for index -- and,
since round 4, for TRAINING at that precision.

The reference computes the whole step in fp32 (``accelerator.autocast()`` is a no-op with empty
``accelerate_kwargs``, ct_clip/CTCLIPTrainer.py:210,216,342).  The default image tower runs its
GEMMs and attention on bf16 operands (~1e-2 relative token error before the VQ), which flips the
cosine argmax of ct_clip/ctvit.py:427 on ~2 % of tokens whose top-2 margin is small (SURVEY 8(c)
counts only flips below a 1e-6 margin as ties).  ``set_vit_precision('f32')`` switches the forward
of the tower's autograd Functions (functional.PatchEmbedFn / ViTLayerFn / ImageProjFn) to:

  * patchify + LayerNorm(4000) in f32 (``ctclip_patch_ln_f32``), then ``to_patch_emb``'s Linear
    and LayerNorm(512) in f32 (ctvit.py:169-174);
  * per layer: PEG (``ctclip_peg_fwd_f32``), bias-less LN, to_q / to_kv, l2norm * scale, cosine
    attention with the CPB bias (``ctclip_attn_fwd_f32``), to_out + residual, FF LayerNorm,
    FF1 + GEGLU, FF2 + residual (attention.py:56-84,127-181,39-52,311-333); norm_out;
  * every Linear on the f32 MFMA GEMM ``ctclip_sgemm_tn`` (v_mfma_f32_16x16x4_f32: one f32 fma chain
    per output, ascending k), the 294,912-wide ``to_visual_latent`` on ``ctclip_sgemm``;
  * the VQ unchanged (its f32 re-score already returns the exact f32 argmax of its input tokens).

Each Function saves the bf16 copies its backward kernels read, so ``CTClipTrainer.train_step``
runs in this mode too: exact-f32 forward (the SURVEY 8(c) contract on the loss the step
differentiates), bf16 backward (gradients are not in the tolerance, as for BERT's hi / lo split
weights).  Cost: DESIGN.md §5.1 and bench.py's ``precise_f32_tower`` entry.

``set_vit_precision('split')`` (round 6) keeps that structure but runs every Linear on the split-fp16
x3 GEMM instead of the f32 MFMA one (gemm256.hip, ctclip_gemm_args.A_lo / B_lo): each operand is an
fp16 (hi, lo) pair -- hi = fp16(x), lo = fp16(x - hi), ~22 mantissa bits -- written by its producer
(patch LayerNorm, f32-tap PEG, the LayerNorms, the x3 GEGLU epilogue), and every K-step runs
Ah Bh + Ah Bl + Al Bh into one f32 accumulator: 3x the fp16 MFMA work instead of f32 MFMA at 1/16 of
the rate.  tools/vit_precision.py prices it on the CPU restatement (sites 's:' / 'S:'): pre-VQ token error
1.2e-6 and 0 flips at base size, against 2.8e-6 for the f32 mode.  Cost: bench.py's
``precise_split_tower`` entry."""
from __future__ import annotations

_MODE = {'vit': 'bf16'}


MODES = ('bf16', 'f32', 'split')


def set_vit_precision(mode):
    """'bf16' (default: 16-bit MFMA kernels, forward + backward), 'f32' (exact-f32 image-tower
    forward, bf16 backward) or 'split' (the f32 mode on split-fp16 x3 GEMMs).  Returns the previous
    mode."""
    if mode not in MODES:
        raise ValueError(mode)
    old = _MODE['vit']
    _MODE['vit'] = mode
    return old


def vit_precision():
    return _MODE['vit']


class vit_precision_scope:
    """``with vit_precision_scope('f32'): ...`` -- the mode inside, the previous one after."""

    def __init__(self, mode):
        self.mode = mode

    def __enter__(self):
        self.old = set_vit_precision(self.mode)
        return self

    def __exit__(self, *exc):
        set_vit_precision(self.old)
        return False


def encode_tokens_f32(vt, video, trace=None):
    """``CTViT.encode_tokens`` in the f32 mode: (z f32 [M, D], z bf16, geometry)."""
    with vit_precision_scope('f32'):
        return vt.encode_tokens(video, trace)
