"""Name-seeded weight recipe + synthetic-input recipe — TEST INFRASTRUCTURE ONLY.

Both the golden-fixture generator (which loads these weights into the reference's own
modules) and the parity tests (which load them into the oracle and into the HIP build)
call ``make_state_dict``, so every side sees bit-identical fp32 weights without
committing hundreds of MB of checkpoints.  Key layout = ``CTCLIP.state_dict()`` of the
reference (``ct_clip/ct_clip.py:587-597``; CTViT built with ``use_vgg_and_gan=False``,
``ct_clip/ctvit.py:198-219``), VQ buffers as restated in ``ctclip_oracle.vq_forward``.
"""
from __future__ import annotations

import zlib
from collections import OrderedDict

import torch

from .ctclip_oracle import ClipConfig, ViTConfig, BertConfig


def _ln_keys(p, d, out, affine_bias=True, buffer_beta=False):
    out[p + ('weight' if affine_bias else 'gamma')] = ('ln_w', (d,))
    if affine_bias:
        out[p + 'bias'] = ('ln_b', (d,))
    if buffer_beta:
        out[p + 'beta'] = ('zeros', (d,))


def vit_keys(cfg: ViTConfig, p='visual_transformer.'):
    k = OrderedDict()
    d, pd = cfg.dim, cfg.patch_dim
    ff = cfg.ff_inner
    inner = cfg.dim_head * cfg.heads
    pdf = cfg.channels * cfg.patch_size * cfg.patch_size
    k[p + 'spatial_rel_pos_bias.net.0.0.weight'] = ('lin', (d, 2))
    k[p + 'spatial_rel_pos_bias.net.0.0.bias'] = ('bias', (d,))
    for li in range(1, cfg.cpb_layers):
        k[p + f'spatial_rel_pos_bias.net.{li}.0.weight'] = ('lin', (d, d))
        k[p + f'spatial_rel_pos_bias.net.{li}.0.bias'] = ('bias', (d,))
    k[p + f'spatial_rel_pos_bias.net.{cfg.cpb_layers}.weight'] = ('lin', (cfg.heads, d))
    k[p + f'spatial_rel_pos_bias.net.{cfg.cpb_layers}.bias'] = ('bias', (cfg.heads,))
    k[p + 'to_patch_emb_first_frame.1.weight'] = ('ln_w', (pdf,))
    k[p + 'to_patch_emb_first_frame.1.bias'] = ('ln_b', (pdf,))
    k[p + 'to_patch_emb_first_frame.2.weight'] = ('lin', (d, pdf))
    k[p + 'to_patch_emb_first_frame.2.bias'] = ('bias', (d,))
    k[p + 'to_patch_emb_first_frame.3.weight'] = ('ln_w', (d,))
    k[p + 'to_patch_emb_first_frame.3.bias'] = ('ln_b', (d,))
    k[p + 'to_patch_emb.1.weight'] = ('ln_w', (pd,))
    k[p + 'to_patch_emb.1.bias'] = ('ln_b', (pd,))
    k[p + 'to_patch_emb.2.weight'] = ('lin', (d, pd))
    k[p + 'to_patch_emb.2.bias'] = ('bias', (d,))
    k[p + 'to_patch_emb.3.weight'] = ('ln_w', (d,))
    k[p + 'to_patch_emb.3.bias'] = ('ln_b', (d,))
    for stack, depth in (('enc_spatial_transformer', cfg.spatial_depth),
                         ('enc_temporal_transformer', cfg.temporal_depth)):
        sp = f'{p}{stack}.'
        for i in range(depth):
            lp = f'{sp}layers.{i}.'
            k[lp + '0.dsconv.weight'] = ('conv', (d, 1, 3, 3, 3))
            k[lp + '0.dsconv.bias'] = ('bias', (d,))
            k[lp + '1.null_kv'] = ('zeros', (cfg.heads, 0, cfg.dim_head))
            k[lp + '1.q_scale'] = ('ln_w', (cfg.dim_head,))
            k[lp + '1.k_scale'] = ('ln_w', (cfg.dim_head,))
            k[lp + '1.norm.gamma'] = ('ln_w', (d,))
            k[lp + '1.norm.beta'] = ('zeros', (d,))
            k[lp + '1.context_norm.gamma'] = ('ln_w', (d,))
            k[lp + '1.context_norm.beta'] = ('zeros', (d,))
            k[lp + '1.to_q.weight'] = ('lin', (inner, d))
            k[lp + '1.to_kv.weight'] = ('lin', (2 * inner, d))
            k[lp + '1.to_out.weight'] = ('lin', (d, inner))
            k[lp + '3.0.weight'] = ('ln_w', (d,))
            k[lp + '3.0.bias'] = ('ln_b', (d,))
            k[lp + '3.1.weight'] = ('lin', (2 * ff, d))
            k[lp + '3.4.weight'] = ('lin', (d, ff))
        k[sp + 'norm_out.gamma'] = ('ln_w', (d,))
        k[sp + 'norm_out.beta'] = ('zeros', (d,))
    k[p + 'vq._codebook.initted'] = ('ones', (1,))
    k[p + 'vq._codebook.cluster_size'] = ('zeros', (1, cfg.codebook_size))
    k[p + 'vq._codebook.embed'] = ('codebook', (1, cfg.codebook_size, d))
    k[p + 'to_pixels_first_frame.0.weight'] = ('lin', (pdf, d))
    k[p + 'to_pixels_first_frame.0.bias'] = ('bias', (pdf,))
    k[p + 'to_pixels.0.weight'] = ('lin', (pd, d))
    k[p + 'to_pixels.0.bias'] = ('bias', (pd,))
    return k


def bert_keys(cfg: BertConfig, p='text_transformer.'):
    k = OrderedDict()
    h = cfg.hidden
    k[p + 'embeddings.word_embeddings.weight'] = ('emb', (cfg.vocab_size, h))
    k[p + 'embeddings.position_embeddings.weight'] = ('emb', (cfg.max_position, h))
    k[p + 'embeddings.token_type_embeddings.weight'] = ('emb', (cfg.type_vocab, h))
    k[p + 'embeddings.LayerNorm.weight'] = ('ln_w', (h,))
    k[p + 'embeddings.LayerNorm.bias'] = ('ln_b', (h,))
    for i in range(cfg.layers):
        lp = f'{p}encoder.layer.{i}.'
        for n in ('query', 'key', 'value'):
            k[lp + f'attention.self.{n}.weight'] = ('lin', (h, h))
            k[lp + f'attention.self.{n}.bias'] = ('bias', (h,))
        k[lp + 'attention.output.dense.weight'] = ('lin', (h, h))
        k[lp + 'attention.output.dense.bias'] = ('bias', (h,))
        k[lp + 'attention.output.LayerNorm.weight'] = ('ln_w', (h,))
        k[lp + 'attention.output.LayerNorm.bias'] = ('ln_b', (h,))
        k[lp + 'intermediate.dense.weight'] = ('lin', (cfg.intermediate, h))
        k[lp + 'intermediate.dense.bias'] = ('bias', (cfg.intermediate,))
        k[lp + 'output.dense.weight'] = ('lin', (h, cfg.intermediate))
        k[lp + 'output.dense.bias'] = ('bias', (h,))
        k[lp + 'output.LayerNorm.weight'] = ('ln_w', (h,))
        k[lp + 'output.LayerNorm.bias'] = ('ln_b', (h,))
    k[p + 'pooler.dense.weight'] = ('lin', (h, h))
    k[p + 'pooler.dense.bias'] = ('bias', (h,))
    return k


def clip_keys(cfg: ClipConfig):
    k = OrderedDict()
    k.update(bert_keys(cfg.bert))
    k.update(vit_keys(cfg.vit))
    k['to_text_latent.weight'] = ('lin', (cfg.dim_latent, cfg.dim_text))
    k['to_visual_latent.weight'] = ('lin', (cfg.dim_latent, cfg.dim_image))
    k['to_text_latent_extra.weight'] = ('lin', (cfg.dim_latent, cfg.dim_text))
    k['to_visual_latent_extra.weight'] = ('lin', (cfg.dim_latent, cfg.dim_image))
    k['temperature'] = ('temp', ())
    return k


def _make(kind, shape, gen):
    if kind == 'zeros':
        return torch.zeros(shape)
    if kind == 'ones':
        return torch.ones(shape)
    if kind == 'temp':
        return torch.tensor(1.0)
    r = torch.randn(shape, generator=gen)
    if kind == 'ln_w':
        return 1.0 + 0.1 * r
    if kind == 'ln_b':
        return 0.05 * r
    if kind == 'bias':
        return 0.02 * r
    if kind == 'lin':
        return r / (shape[1] ** 0.5)
    if kind == 'conv':
        return r / (27 ** 0.5)
    if kind == 'emb':
        return 0.5 * r
    if kind == 'codebook':
        return torch.nn.functional.normalize(r, dim=-1)
    raise ValueError(kind)


def make_state_dict(cfg: ClipConfig, seed: int = 0, skip=()):
    """Deterministic fp32 state_dict: every tensor seeded by crc32(key) ^ seed."""
    sd = OrderedDict()
    for key, (kind, shape) in clip_keys(cfg).items():
        if key in skip:
            continue
        g = torch.Generator().manual_seed((zlib.crc32(key.encode()) ^ seed) & 0x7FFFFFFF)
        sd[key] = _make(kind, shape, g).to(torch.float32).contiguous()
    return sd


# ----------------------------------------------------------------------------- inputs
def make_hu(batch, cfg: ViTConfig, seed=1234, lo=-1200, hi=1201):
    """Synthetic int16 HU volume: randint(-1200, 1201), seeded."""
    g = torch.Generator().manual_seed(seed)
    return torch.randint(lo, hi, (batch, cfg.channels, cfg.frames, cfg.image_size, cfg.image_size),
                         generator=g, dtype=torch.int16)


def make_text(batch, length, vocab, seed=4321, ragged=False):
    """Token ids: CLS=2 first, uniform ids in [5, vocab), SEP=3 last; optional ragged
    lengths with pad id 0."""
    g = torch.Generator().manual_seed(seed)
    ids = torch.randint(5, vocab, (batch, length), generator=g)
    mask = torch.ones(batch, length, dtype=torch.long)
    lens = [length] * batch
    if ragged:
        lens = torch.randint(max(2, length // 4), length + 1, (batch,), generator=g).tolist()
        lens[0] = length
    for b, n in enumerate(lens):
        ids[b, 0] = 2
        ids[b, n - 1] = 3
        ids[b, n:] = 0
        mask[b, n:] = 0
    return ids, mask


def make_projector(input_dim=512, feature_dim=512, seed=0):
    """VisionFeatureExtractor.feature_projector (ctpa_report/vqa_meditron.py:42-46):
    Linear(input_dim, feature_dim) + LayerNorm(feature_dim) (+ GELU), name-seeded like the rest."""
    keys = OrderedDict([('feature_projector.0.weight', ('lin', (feature_dim, input_dim))),
                        ('feature_projector.0.bias', ('bias', (feature_dim,))),
                        ('feature_projector.1.weight', ('ln_w', (feature_dim,))),
                        ('feature_projector.1.bias', ('ln_b', (feature_dim,)))])
    sd = OrderedDict()
    for key, (kind, shape) in keys.items():
        g = torch.Generator().manual_seed((zlib.crc32(key.encode()) ^ seed) & 0x7FFFFFFF)
        sd[key] = _make(kind, shape, g).to(torch.float32).contiguous()
    return sd
