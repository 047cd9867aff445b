"""VisionFeatureExtractor (ctpa_report/vqa_meditron.py:26-131) on HIP kernels.

Signature kept: ``VisionFeatureExtractor(vision_encoder, feature_dim=512, device=None)`` and
``forward(x) -> (b, feature_dim)``.  As shipped, the reference's forward always falls back to
``torch.randn`` (its spatial-transformer call lacks ``video_shape``, attention.py:65); this build
implements the intended deterministic path: to_patch_emb -> spatial transformer (with
video_shape and the CPB bias) -> mean over all tokens -> Linear + LayerNorm + GELU
(input_dim = 512 via the reference's own fallback, vqa_meditron.py:52-89).
"""
from __future__ import annotations

import torch
from torch import nn

from . import functional as Fn
from . import kernels as K


class VisionFeatureExtractor(nn.Module):
    def __init__(self, vision_encoder, feature_dim=512, device=None):
        super().__init__()
        self.device = device or torch.device('cuda')
        self.vision_encoder = vision_encoder.to(self.device)
        self.input_dim = vision_encoder.dim
        self.feature_projector = nn.Sequential(nn.Linear(self.input_dim, feature_dim), nn.LayerNorm(feature_dim),
                                               nn.GELU()).to(self.device)

    @torch.no_grad()
    def forward(self, x):
        ve = self.vision_encoder
        if x.dtype != torch.int16:
            x = x.to(self.device).float()
        else:
            x = x.to(self.device)
        if x.ndim == 4:
            x = x.unsqueeze(2)
        B, C, F, H, W = x.shape
        pe = ve.to_patch_emb
        xf, xb = Fn.PatchEmbedFn.apply(x.contiguous(), pe[1].weight, pe[1].bias, pe[2].weight, pe[2].bias,
                                       pe[3].weight, pe[3].bias, ve.temporal_patch_size, ve.patch_size[0],
                                       x.dtype == torch.int16, ve._offsets(x.shape, x.device))
        hg, wg = ve.patch_height_width
        T = F // ve.temporal_patch_size
        geo = Fn.Geo(B, T, hg, wg, ve.heads, ve.dim_head, 0)
        bias_u = ve.spatial_rel_pos_bias(hg, wg)
        yf, _ = ve.enc_spatial_transformer.run(xf, xb, geo, bias_u)
        pooled = K.colsum_rows_mean(yf, B)                     # (B, D): mean over t*h*w tokens
        lin, ln = self.feature_projector[0], self.feature_projector[1]
        h = K.slinear(pooled, lin.weight, lin.bias)
        hb, hf, _, _ = K.layernorm_fwd(h, ln.weight, ln.bias, ln.eps, out_bf16=False, out_f32=True)
        return K.gelu_f32(hf)
