"""VisionFeatureExtractor (ctpa_report/vqa_meditron.py:26-131) on HIP kernels (configs[4]).

Signature kept: ``VisionFeatureExtractor(vision_encoder, feature_dim=512, device=None)`` and
``forward(x) -> (b, feature_dim)``.

* ``input_dim``: the reference probes the encoder with a (1, 1, pt, H/p, W/p) sample
  (``_safe_infer_input_dimension``, :52-89).  That probe always fails -- to_patch_emb's
  rearrange needs H/p to be a multiple of p, and even then the spatial transformer call has no
  ``video_shape`` -- so the reference always takes ``fallback_dim = 512``.  This build takes
  512 directly (``_safe_infer_input_dimension`` below returns it without running the probe).
* ``forward``: as shipped, the reference's spatial-transformer call (:107) omits ``video_shape``,
  PEG's assert (ct_clip/attention.py:65) raises, and the forward returns ``torch.randn`` (:125-127).
  This build runs the intended path with that one repair: to_patch_emb -> spatial transformer
  with video_shape and, like the reference call, no attention bias (``position_bias=True`` adds
  the CPB bias CTViT.encode uses) -> mean over every token (:114-117) -> Linear + LayerNorm +
  GELU (:42-46, :120).  It returns (b, feature_dim) also for b = 1, where the reference's
  ``.squeeze()`` would give (feature_dim,).  Errors raise instead of returning random features.
"""
from __future__ import annotations

import torch
from torch import nn

from . import functional as Fn
from . import kernels as K


class VisionFeatureExtractor(nn.Module):
    def __init__(self, vision_encoder, feature_dim=512, device=None, position_bias=False):
        super().__init__()
        self.device = device or torch.device('cuda')
        self.vision_encoder = vision_encoder.to(self.device)
        self.position_bias = position_bias
        self.input_dim = self._safe_infer_input_dimension()
        self.feature_projector = nn.Sequential(nn.Linear(self.input_dim, feature_dim), nn.LayerNorm(feature_dim),
                                               nn.GELU()).to(self.device)

    def _safe_infer_input_dimension(self, fallback_dim=512):
        """vqa_meditron.py:52-89: the probe never succeeds (see module docstring) -> fallback_dim."""
        return fallback_dim

    @torch.no_grad()
    def forward(self, x):
        ve = self.vision_encoder
        if ve.dim != self.input_dim:
            raise ValueError(f'vision encoder dim {ve.dim} != feature_projector input {self.input_dim} '
                             '(the reference returns torch.randn features here)')
        x = x.to(self.device)
        if x.dtype != torch.int16:
            x = x.float()
        if x.ndim == 4:
            x = x.unsqueeze(2)
        B, C, F, H, W = x.shape
        if (H, W) != tuple(ve.image_size) or F % ve.temporal_patch_size:
            raise ValueError(f'volume {tuple(x.shape)} does not tile into {ve.temporal_patch_size} x '
                             f'{ve.patch_size[0]} x {ve.patch_size[0]} patches of a {ve.image_size} image')
        pe = ve.to_patch_emb
        xf, xb = Fn.PatchEmbedFn.apply(x.contiguous(), pe[1].weight, pe[1].bias, pe[2].weight, pe[2].bias,
                                       pe[3].weight, pe[3].bias, ve.temporal_patch_size, ve.patch_size[0],
                                       x.dtype == torch.int16, ve._offsets(x.shape, x.device))
        hg, wg = ve.patch_height_width
        T = F // ve.temporal_patch_size
        geo = Fn.Geo(B, T, hg, wg, ve.heads, ve.dim_head, 0)
        bias_u = ve.spatial_rel_pos_bias(hg, wg) if self.position_bias else None
        yf, _ = ve.enc_spatial_transformer.run(xf, xb, geo, bias_u)
        pooled = K.colsum_rows_mean(yf, B)                     # (B, D): mean over t*h*w tokens
        lin, ln = self.feature_projector[0], self.feature_projector[1]
        h = K.slinear(pooled, lin.weight, lin.bias)
        hb, hf, _, _ = K.layernorm_fwd(h, ln.weight, ln.bias, ln.eps, out_bf16=False, out_f32=True)
        return K.gelu_f32(hf)
