"""CPU fp32 restatement of the CT-CLIP contrastive step — TEST INFRASTRUCTURE ONLY.

This module is the parity oracle for the MI355X build.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it,
and only as the checker / the timed CPU baseline.  The product package
(``ctpa-clip_amd/ctclip_mi355x``) never imports it and fails loudly when its
HIP library is missing.

It is a functional restatement (plain torch fp32 eager on CPU) of the reference's
hot path, written from scratch and driven by a ``state_dict`` that uses the
reference's own key layout (``ct_clip/ct_clip.py:587-597``).  Each function cites
the reference file:line it restates (paths relative to CTPA_CLIP/).

Parity pinning: ``tests/golden/make_golden.py`` imports the reference modules in
this container (with import-time stubs for deps missing offline: beartype,
torchvision, vector_quantize_pytorch) and writes fixtures under ``tests/golden``;
``tests/test_oracle_golden.py`` checks this restatement against them.  The
vector-quantiser arithmetic lives in the third-party ``vector_quantize_pytorch==1.1.2``
(``requirements.txt:9``), which is neither vendored nor installed: its restatement
below (``vq_forward``) is *parity unpinned* beyond "indices are the argmax of the
cosine similarity" — see DESIGN.md §Oracle.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import torch
import torch.nn.functional as F


# ----------------------------------------------------------------------------- configs
@dataclass(frozen=True)
class ViTConfig:
    """CTViT constructor arguments (``ct_clip/pretrained_model.py:17-27``)."""
    dim: int = 512
    codebook_size: int = 8192
    image_size: int = 480
    patch_size: int = 20
    temporal_patch_size: int = 10
    spatial_depth: int = 4
    temporal_depth: int = 4
    dim_head: int = 32
    heads: int = 8
    channels: int = 1
    frames: int = 240          # input depth D (``ct_clip/data.py:155``)
    cpb_layers: int = 2        # ContinuousPositionBias default (``ct_clip/attention.py:238``)
    vq_decay: float = 0.8      # vector_quantize_pytorch default (unpinned)

    @property
    def grid(self):
        return self.image_size // self.patch_size

    @property
    def t_tokens(self):
        return self.frames // self.temporal_patch_size

    @property
    def patch_dim(self):
        return self.channels * self.temporal_patch_size * self.patch_size * self.patch_size

    @property
    def ff_inner(self):
        # ``ct_clip/attention.py:45``: int(mult * 2/3 * dim), mult = 4
        return int(4 * (2 / 3) * self.dim)


@dataclass(frozen=True)
class BertConfig:
    """BERT-base as used by CXR-BERT-specialized (``ct_clip/pretrained_model.py:9``)."""
    vocab_size: int = 30522
    hidden: int = 768
    layers: int = 12
    heads: int = 12
    intermediate: int = 3072
    max_position: int = 512
    type_vocab: int = 2
    eps: float = 1e-12
    pad_id: int = 0     # word table padding_idx (transformers BertEmbeddings, pad_token_id)


@dataclass(frozen=True)
class ClipConfig:
    vit: ViTConfig = field(default_factory=ViTConfig)
    bert: BertConfig = field(default_factory=BertConfig)
    dim_latent: int = 512

    @property
    def dim_text(self):
        return self.bert.hidden

    @property
    def dim_image(self):
        # ``ct_clip/ct_clip.py:724,740``: mean over t, then flatten (h, w, d)
        return self.vit.grid * self.vit.grid * self.vit.dim


BASE = ClipConfig()
TINY = ClipConfig(
    vit=ViTConfig(dim=64, codebook_size=128, image_size=32, patch_size=8, temporal_patch_size=4,
                  spatial_depth=2, temporal_depth=2, dim_head=16, heads=4, frames=32),
    bert=BertConfig(vocab_size=1000, hidden=64, layers=2, heads=4, intermediate=256, max_position=64),
    dim_latent=32,
)


# ----------------------------------------------------------------------------- input
def normalize_hu(hu: torch.Tensor) -> torch.Tensor:
    """int16 HU -> f32 in [-1, 1] (``ct_clip/data.py:150-152``).

    ``np.clip(x, -1000, 1000)`` then ``(x / 1000).astype(np.float32)``: the reference divides
    in f64 and casts; an f32 division by 1000.f is bit-identical for every int16 value
    (checked exhaustively in tests/test_oracle_golden.py)."""
    return hu.to(torch.float32).clamp(-1000.0, 1000.0) / 1000.0


# ----------------------------------------------------------------------------- CTViT pieces
def _ln(x, w, b, eps=1e-5):
    return F.layer_norm(x, x.shape[-1:], w, b, eps)


def patch_embed(sd, p, video, cfg: ViTConfig):
    """``CTViT.to_patch_emb`` (``ct_clip/ctvit.py:169-174``): rearrange
    'b c (t pt) (h p1) (w p2) -> b t h w (c pt p1 p2)', LayerNorm(4000), Linear, LayerNorm(512)."""
    b, c, f, hh, ww = video.shape
    pt, ps = cfg.temporal_patch_size, cfg.patch_size
    t, h, w = f // pt, hh // ps, ww // ps
    x = video.reshape(b, c, t, pt, h, ps, w, ps)
    x = x.permute(0, 2, 4, 6, 1, 3, 5, 7).reshape(b, t, h, w, c * pt * ps * ps)
    x = _ln(x, sd[p + 'to_patch_emb.1.weight'], sd[p + 'to_patch_emb.1.bias'])
    x = F.linear(x, sd[p + 'to_patch_emb.2.weight'], sd[p + 'to_patch_emb.2.bias'])
    x = _ln(x, sd[p + 'to_patch_emb.3.weight'], sd[p + 'to_patch_emb.3.bias'])
    return x


def cpb_rel_pos(h, w):
    """Log-spaced relative positions of an h x w grid (``ct_clip/attention.py:257-269``)."""
    pos = torch.stack(torch.meshgrid(torch.arange(h), torch.arange(w), indexing='ij'))
    grid = pos.reshape(2, -1).t()                                   # (h*w, 2)
    rel = grid[:, None, :] - grid[None, :, :]                       # (i, j, 2)
    return torch.sign(rel) * torch.log(rel.abs() + 1)               # float


def cpb_forward(sd, p, h, w, layers=2):
    """``ContinuousPositionBias.forward`` (``ct_clip/attention.py:257-276``): MLP over the
    relative positions in fp32, LeakyReLU(0.1) between layers, output (heads, i, j)."""
    x = cpb_rel_pos(h, w).to(torch.float32)
    for li in range(layers):
        x = F.leaky_relu(F.linear(x, sd[f'{p}net.{li}.0.weight'], sd[f'{p}net.{li}.0.bias']), 0.1)
    x = F.linear(x, sd[f'{p}net.{layers}.weight'], sd[f'{p}net.{layers}.bias'])
    return x.permute(2, 0, 1)


def peg_forward(sd, p, x, shape):
    """``PEG.forward`` with causal=True (``ct_clip/attention.py:56-84``; ``ct_clip/ctvit.py:183``).

    x is (N, n, d) and is *raw-reshaped* to (b, t, h, w, d) (``attention.py:69-70``); in the
    temporal transformer x is laid out '(b h w) t d', so the conv runs on that scrambled view —
    reproduced here exactly because we use the same reshape."""
    orig = x.shape
    v = x.reshape(*shape, -1)                                       # (b, t, h, w, d)
    v = v.permute(0, 4, 1, 2, 3)                                    # b d t h w
    v = F.pad(v, (1, 1, 1, 1, 2, 0), value=0.0)
    v = F.conv3d(v, sd[p + 'dsconv.weight'], sd[p + 'dsconv.bias'], groups=v.shape[1])
    v = v.permute(0, 2, 3, 4, 1)
    return v.reshape(orig)


def attention_forward(sd, p, x, heads, dim_head, attn_bias=None):
    """``Attention.forward`` (``ct_clip/attention.py:127-181``), self-attention, no mask,
    num_null_kv = 0.  K/V come from the *un-normalised* x (``:139-143``)."""
    n_b, n, _ = x.shape
    kv_input = x
    xn = _ln(x, sd[p + 'norm.gamma'], sd[p + 'norm.beta'])
    q = F.linear(xn, sd[p + 'to_q.weight'])
    k, v = F.linear(kv_input, sd[p + 'to_kv.weight']).chunk(2, dim=-1)

    def split(t):
        return t.reshape(n_b, n, heads, dim_head).permute(0, 2, 1, 3)
    q, k, v = split(q), split(k), split(v)
    q = F.normalize(q, dim=-1) * sd[p + 'q_scale']
    k = F.normalize(k, dim=-1) * sd[p + 'k_scale']
    sim = torch.einsum('bhid,bhjd->bhij', q, k) * 8.0
    if attn_bias is not None:
        sim = sim + attn_bias
    attn = sim.softmax(dim=-1)
    out = torch.einsum('bhij,bhjd->bhid', attn, v)
    out = out.permute(0, 2, 1, 3).reshape(n_b, n, heads * dim_head)
    return F.linear(out, sd[p + 'to_out.weight'])


def ff_forward(sd, p, x):
    """``FeedForward`` (``ct_clip/attention.py:39-52``): LayerNorm -> Linear -> GEGLU -> Linear."""
    x = _ln(x, sd[p + '0.weight'], sd[p + '0.bias'])
    x = F.linear(x, sd[p + '1.weight'])
    a, gate = x.chunk(2, dim=-1)
    x = F.gelu(gate) * a
    return F.linear(x, sd[p + '4.weight'])


def transformer_forward(sd, p, x, depth, heads, dim_head, video_shape, attn_bias=None):
    """``Transformer.forward`` (``ct_clip/attention.py:311-333``)."""
    for i in range(depth):
        lp = f'{p}layers.{i}.'
        x = peg_forward(sd, lp + '0.', x, video_shape) + x
        x = attention_forward(sd, lp + '1.', x, heads, dim_head, attn_bias) + x
        x = ff_forward(sd, lp + '3.', x) + x
    return _ln(x, sd[p + 'norm_out.gamma'], sd[p + 'norm_out.beta'])


def ctvit_encode(sd, p, tokens, cfg: ViTConfig, trace=None):
    """``CTViT.encode`` (``ct_clip/ctvit.py:306-331``)."""
    b, t, h, w, d = tokens.shape
    video_shape = (b, t, h, w)
    x = tokens.reshape(b * t, h * w, d)
    bias = cpb_forward(sd, p + 'spatial_rel_pos_bias.', h, w, cfg.cpb_layers)
    if trace is not None:
        trace['cpb'] = bias
    x = transformer_forward(sd, p + 'enc_spatial_transformer.', x, cfg.spatial_depth, cfg.heads,
                            cfg.dim_head, video_shape, bias)
    x = x.reshape(b, t, h, w, d)
    if trace is not None:
        trace['spatial_out'] = x
    x = x.permute(0, 2, 3, 1, 4).reshape(b * h * w, t, d)
    x = transformer_forward(sd, p + 'enc_temporal_transformer.', x, cfg.temporal_depth, cfg.heads,
                            cfg.dim_head, video_shape, None)
    x = x.reshape(b, h, w, t, d).permute(0, 3, 1, 2, 4)
    if trace is not None:
        trace['temporal_out'] = x
    return x


# ----------------------------------------------------------------------------- VQ (unpinned)
def vq_forward(x, embed, cluster_size, training, decay=0.8, force_ind=None):
    """Cosine-similarity VectorQuantize, restated from the published algorithm of
    ``vector_quantize_pytorch==1.1.2`` (third-party; called at ``ct_clip/ctvit.py:187,427``).

    x (..., d) -> (quantized, indices, new_embed, new_cluster_size).
    * l2norm(x) @ embedᵀ, argmax -> indices; quantize = embed[indices] (pre-update codebook)
    * training: EMA update with decay (bins, l2-normalised per-code mean, zero bins keep
      the old code); straight-through estimator x + (q - x).detach().
    PARITY UNPINNED beyond the argmax: see module docstring."""
    shape = x.shape
    flat = F.normalize(x.reshape(-1, shape[-1]).float(), dim=-1)
    emb = embed.reshape(-1, shape[-1])
    dist = flat @ emb.t()
    ind = dist.argmax(dim=-1) if force_ind is None else force_ind.reshape(-1).to(torch.int64)
    q = emb[ind]
    new_embed, new_cs = embed, cluster_size
    if training:
        with torch.no_grad():
            onehot = F.one_hot(ind, emb.shape[0]).to(flat.dtype)
            bins = onehot.sum(0)
            new_cs = cluster_size * decay + bins.reshape(cluster_size.shape) * (1 - decay)
            zero = bins == 0
            bins_c = bins.masked_fill(zero, 1.0)
            esum = onehot.t() @ flat.detach()
            en = F.normalize(esum / bins_c[:, None], dim=-1)
            en = torch.where(zero[:, None], emb, en)
            new_embed = (emb * decay + en * (1 - decay)).reshape(embed.shape)
        q = x.reshape(-1, shape[-1]) + (q - x.reshape(-1, shape[-1])).detach()
    return q.reshape(shape), ind.reshape(shape[:-1]), new_embed, new_cs


def ctvit_forward(sd, p, video, cfg: ViTConfig, training, trace=None, force_ind=None):
    """``CTViT.forward(video, return_encoded_tokens=True)`` (``ct_clip/ctvit.py:377-436``).
    Returns (tokens (b,t,h,w,d), indices (b, t*h*w), new_embed, new_cluster_size).
    ``force_ind`` (test hook) replaces the argmax so near-tie index flips of a reduced-precision
    implementation can be separated from everything downstream of the quantiser."""
    tokens = patch_embed(sd, p, video, cfg)
    if trace is not None:
        trace['patch_emb'] = tokens
    b, t, h, w, d = tokens.shape
    x = ctvit_encode(sd, p, tokens, cfg, trace)
    x = x.reshape(b, t * h * w, d)
    q, ind, ne, ncs = vq_forward(x, sd[p + 'vq._codebook.embed'], sd[p + 'vq._codebook.cluster_size'],
                                 training, cfg.vq_decay, force_ind)
    return q.reshape(b, t, h, w, d), ind, ne, ncs


def ctvit_decode(sd, p, tokens, cfg: ViTConfig):
    """``CTViT.decode`` (``ct_clip/ctvit.py:333-375``): the ENCODER's temporal then spatial
    transformers run again on the quantised tokens (temporal on '(b h w) t d' with the same raw-
    reshape PEG view, spatial with the CPB bias), then ``to_pixels`` (``:194-197``): Linear(dim ->
    c*pt*p1*p2) and 'b t h w (c pt p1 p2) -> b c (t pt) (h p1) (w p2)'."""
    b, t, h, w, d = tokens.shape
    video_shape = (b, t, h, w)
    x = tokens.permute(0, 2, 3, 1, 4).reshape(b * h * w, t, d)
    x = transformer_forward(sd, p + 'enc_temporal_transformer.', x, cfg.temporal_depth, cfg.heads,
                            cfg.dim_head, video_shape, None)
    x = x.reshape(b, h, w, t, d).permute(0, 3, 1, 2, 4).reshape(b * t, h * w, d)
    bias = cpb_forward(sd, p + 'spatial_rel_pos_bias.', h, w, cfg.cpb_layers)
    x = transformer_forward(sd, p + 'enc_spatial_transformer.', x, cfg.spatial_depth, cfg.heads,
                            cfg.dim_head, video_shape, bias)
    y = F.linear(x.reshape(b, t, h, w, d), sd[p + 'to_pixels.0.weight'], sd[p + 'to_pixels.0.bias'])
    c, pt, ps = cfg.channels, cfg.temporal_patch_size, cfg.patch_size
    y = y.reshape(b, t, h, w, c, pt, ps, ps).permute(0, 4, 1, 5, 2, 6, 3, 7)
    return y.reshape(b, c, t * pt, h * ps, w * ps)


def ctvit_recon(sd, p, video, cfg: ViTConfig, training, force_ind=None):
    """``CTViT.forward(video, return_recons=True)`` with ``use_vgg_and_gan=False``
    (``ct_clip/ctvit.py:377-451``): patch embed -> encode -> VQ (STE) -> decode ->
    ``F.mse_loss(video, recon)``.  Returns (loss, recon, indices, new_embed, new_cluster_size)."""
    tokens, ind, ne, ncs = ctvit_forward(sd, p, video, cfg, training, None, force_ind)
    recon = ctvit_decode(sd, p, tokens, cfg)
    return F.mse_loss(video, recon), recon, ind, ne, ncs


# ----------------------------------------------------------------------------- BERT
def bert_forward(sd, p, ids, mask, cfg: BertConfig):
    """BERT-base encoder as called at ``ct_clip/ct_clip.py:685-686`` (third-party
    ``transformers.BertModel``; restated: post-LN, GELU-erf, additive -inf-style mask,
    dropout 0).  Returns last_hidden_state (b, L, hidden)."""
    b, L = ids.shape
    pos = torch.arange(L)
    # padding_idx: the pad id's row takes part in the forward but gets no gradient
    x = F.embedding(ids, sd[p + 'embeddings.word_embeddings.weight'], padding_idx=cfg.pad_id) \
        + sd[p + 'embeddings.token_type_embeddings.weight'][0] \
        + sd[p + 'embeddings.position_embeddings.weight'][pos]
    x = _ln(x, sd[p + 'embeddings.LayerNorm.weight'], sd[p + 'embeddings.LayerNorm.bias'], cfg.eps)
    nh, hd = cfg.heads, cfg.hidden // cfg.heads
    add_mask = (1.0 - mask.to(torch.float32))[:, None, None, :] * torch.finfo(torch.float32).min
    for i in range(cfg.layers):
        lp = f'{p}encoder.layer.{i}.'

        def lin(t, name):
            return F.linear(t, sd[lp + name + '.weight'], sd[lp + name + '.bias'])
        q = lin(x, 'attention.self.query').reshape(b, L, nh, hd).transpose(1, 2)
        k = lin(x, 'attention.self.key').reshape(b, L, nh, hd).transpose(1, 2)
        v = lin(x, 'attention.self.value').reshape(b, L, nh, hd).transpose(1, 2)
        s = (q @ k.transpose(-1, -2)) / math.sqrt(hd) + add_mask
        a = s.softmax(-1) @ v
        a = a.transpose(1, 2).reshape(b, L, cfg.hidden)
        x = _ln(lin(a, 'attention.output.dense') + x, sd[lp + 'attention.output.LayerNorm.weight'],
                sd[lp + 'attention.output.LayerNorm.bias'], cfg.eps)
        hmid = F.gelu(lin(x, 'intermediate.dense'))
        x = _ln(lin(hmid, 'output.dense') + x, sd[lp + 'output.LayerNorm.weight'],
                sd[lp + 'output.LayerNorm.bias'], cfg.eps)
    return x


# ----------------------------------------------------------------------------- CT-CLIP head + loss
def clip_latents(sd, enc_text, enc_image):
    """Pool + projections + l2norm (``ct_clip/ct_clip.py:724,740,762-771``)."""
    img = enc_image.mean(dim=1)                          # mean over t
    img = img.reshape(img.shape[0], -1)                  # (b, h*w*d)
    t_lat = F.linear(enc_text[:, 0, :], sd['to_text_latent.weight'])
    i_lat = F.linear(img, sd['to_visual_latent.weight'])
    return F.normalize(t_lat, dim=-1), F.normalize(i_lat, dim=-1)


def infonce(text_latents, image_latents, temperature):
    """Symmetric contrastive loss exactly as ``ct_clip/ct_clip.py:796,845-901`` (no max
    subtraction, log(x + 1e-20), mean over rows, /2)."""
    temp = temperature.exp()
    t2i = text_latents @ image_latents.t() * temp
    i2t = t2i.t()

    def one(s):
        e = s.exp()
        pos = torch.diagonal(e)
        den = e.sum(dim=-1)
        return (-torch.log(pos + 1e-20) + torch.log(den + 1e-20)).mean()
    return (one(t2i) + one(i2t)) / 2


def ctclip_forward(sd, ids, mask, video, cfg: ClipConfig, training=True, trace=None, force_ind=None):
    """``CTCLIP.forward(text, image, return_loss=True)`` (``ct_clip/ct_clip.py:614-901``)
    with MLM / visual-SSL / multiview off (``pretrained_model.py:31-42``).
    Returns dict(loss, text_latents, image_latents, enc_image, indices, new_embed, new_cluster_size)."""
    enc_text = bert_forward(sd, 'text_transformer.', ids, mask, cfg.bert)
    enc_image, ind, ne, ncs = ctvit_forward(sd, 'visual_transformer.', video, cfg.vit, training, trace, force_ind)
    t_lat, i_lat = clip_latents(sd, enc_text, enc_image)
    loss = infonce(t_lat, i_lat, sd['temperature'])
    return dict(loss=loss, text_latents=t_lat, image_latents=i_lat, enc_image=enc_image,
                enc_text=enc_text, indices=ind, new_embed=ne, new_cluster_size=ncs)


def eval_scores(sd, ids, mask, video, cfg: ClipConfig):
    """Eval branch ``einsum('b d, b d -> b') * temp`` (``ct_clip/ct_clip.py:805-807``)."""
    out = ctclip_forward(sd, ids, mask, video, cfg, training=False)
    return (out['text_latents'] * out['image_latents']).sum(-1) * sd['temperature'].exp()


# ----------------------------------------------------------------------------- zero-shot
# ct_clip/ctclip_inference.py:286-290
PATHOLOGIES = ('Medical material', 'Arterial wall calcification', 'Cardiomegaly', 'Pericardial effusion',
               'Coronary artery wall calcification', 'Hiatal hernia', 'Lymphadenopathy', 'Emphysema',
               'Atelectasis', 'Lung nodule', 'Lung opacity', 'Pulmonary Embolism', 'Pleural effusion',
               'Mosaic attenuation pattern', 'Peribronchial thickening', 'Consolidation', 'Bronchiectasis',
               'Interlobular septal thickening')


def zero_shot(sd, ids, mask, video, cfg: ClipConfig, force_ind=None):
    """Zero-shot pathology scoring, the loop of ``ct_clip/ctclip_inference.py:291-318``: for each
    volume (batch 1) and each pathology, the prompt pair ("<p> is present.", "<p> is not
    present.") -- rows (2j, 2j+1) of ``ids`` / ``mask`` -- goes through ``CTCLIP.forward`` in eval
    mode (``einsum('b d, b d -> b') * temp`` with the one image broadcast over the 2 texts,
    ``ct_clip.py:805-807``), then ``softmax(dim=0)`` (``ctclip_inference.py:92-104,312``) and the
    'present' entry is kept (``:315``).  The reference re-encodes the identical volume for every
    pathology; eval mode is deterministic, so the volume is encoded once here.
    Returns (probs [N, P], scores [N, P, 2])."""
    n, P = video.shape[0], ids.shape[0] // 2
    enc_text = bert_forward(sd, 'text_transformer.', ids, mask, cfg.bert)
    temp = sd['temperature'].exp()
    probs, scores = torch.empty(n, P), torch.empty(n, P, 2)
    for v in range(n):
        fi = None if force_ind is None else force_ind[v:v + 1]
        enc_image, _, _, _ = ctvit_forward(sd, 'visual_transformer.', video[v:v + 1], cfg.vit, False, None, fi)
        for j in range(P):
            t_lat, i_lat = clip_latents(sd, enc_text[2 * j:2 * j + 2], enc_image)
            s = (t_lat * i_lat).sum(-1) * temp                     # (2,): the image row broadcasts
            scores[v, j] = s
            probs[v, j] = torch.softmax(s, dim=0)[0]
    return probs, scores


# ----------------------------------------------------------------------------- VQA vision features
VFE_FALLBACK_DIM = 512
# parity config of the extractor: base widths on a reduced 160 x 160 x 40 volume (4 x 8 x 8 tokens)
VFE_VIT = ViTConfig(image_size=160, frames=40, spatial_depth=4, temporal_depth=1)


def vision_features(sd, p, video, cfg: ViTConfig, proj, position_bias=False, trace=None):
    """``VisionFeatureExtractor.forward`` (``ctpa_report/vqa_meditron.py:91-123``) on its intended
    path.  As shipped, the reference's call ``enc_spatial_transformer(spatial_input)`` (``:107``)
    omits ``video_shape``, PEG's assert (``ct_clip/attention.py:65``) raises and the forward returns
    ``torch.randn`` (``:125-127``); the one repair restated here is passing
    ``video_shape = (b, t, h, w)``.  No ``attn_bias`` (the reference call passes none;
    ``position_bias=True`` adds the CPB bias of ``CTViT.encode``, ``ctvit.py:317``).  Then the mean
    over every token (``adaptive_avg_pool3d(..., (1, 1, 1))``, ``:114-117``, over the token grid)
    and ``feature_projector`` = Linear + LayerNorm + GELU(erf) (``:42-46``).
    ``proj`` holds the ``feature_projector.*`` tensors; returns (b, feature_dim)."""
    tokens = patch_embed(sd, p, video, cfg)                         # (b, t, h, w, d)
    b, t, h, w, d = tokens.shape
    x = tokens.reshape(b * t, h * w, d)                             # vqa_meditron.py:134-141
    bias = cpb_forward(sd, p + 'spatial_rel_pos_bias.', h, w, cfg.cpb_layers) if position_bias else None
    x = transformer_forward(sd, p + 'enc_spatial_transformer.', x, cfg.spatial_depth, cfg.heads,
                            cfg.dim_head, (b, t, h, w), bias)
    pooled = x.reshape(b, t * h * w, d).mean(dim=1)
    if trace is not None:
        trace.update(patch_emb=tokens, spatial_out=x.reshape(b, t, h, w, d), pooled=pooled)
    y = F.linear(pooled, proj['feature_projector.0.weight'], proj['feature_projector.0.bias'])
    y = F.layer_norm(y, y.shape[-1:], proj['feature_projector.1.weight'], proj['feature_projector.1.bias'], 1e-5)
    return F.gelu(y)


# ----------------------------------------------------------------------------- weights recipe
def trainable_prefixes():
    """``ct_clip/fine_tuning_ctclip.py:6-14``: only visual_transformer and text_transformer
    train; projections and temperature are frozen."""
    return ('visual_transformer.', 'text_transformer.')
