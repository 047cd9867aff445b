"""VisionFeatureExtractor (configs[4], ctpa_report/vqa_meditron.py:26-131) on the GPU.

* reduced volume (base widths, 160 x 160 x 40 -> 4 x 8 x 8 tokens, 4 spatial layers) against the
  reference's own modules (tests/golden/golden_vfe.safetensors, make_golden.py --vfe):
  patch-embed, spatial-transformer output, pooled tokens and the projected features;
* the full configs[4] volume (1, 1, 240, 480, 480) -> (1, 512) against the oracle's
  vision_features (pinned to the same fixture by tests/test_oracle_golden.py);
* the CPB-bias variant (position_bias=True) against the oracle, and the constructor contract
  (input_dim = the reference's fallback 512)."""
import os

import pytest
import torch

from oracle import ctclip_oracle as O
from oracle import weights as W

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def make_vfe(vit: O.ViTConfig, position_bias=False):
    from ctclip_mi355x.ctvit import CTViT
    from ctclip_mi355x.vqa import VisionFeatureExtractor
    sd = W.make_state_dict(O.ClipConfig(vit=vit, bert=O.TINY.bert, dim_latent=512))
    ve = CTViT(dim=vit.dim, codebook_size=vit.codebook_size, image_size=vit.image_size, patch_size=vit.patch_size,
               temporal_patch_size=vit.temporal_patch_size, spatial_depth=vit.spatial_depth,
               temporal_depth=vit.temporal_depth, dim_head=vit.dim_head, heads=vit.heads)
    p = 'visual_transformer.'
    ve.load_state_dict({k[len(p):]: v for k, v in sd.items() if k.startswith(p)}, strict=True)
    ve.eval()
    fe = VisionFeatureExtractor(ve, feature_dim=512, device=torch.device('cuda'), position_bias=position_bias)
    proj = W.make_projector(512, 512)
    fe.feature_projector.load_state_dict({k[len('feature_projector.'):]: v for k, v in proj.items()}, strict=True)
    return fe, sd, proj


def test_vfe_matches_reference_fixture():
    from safetensors.torch import load_file
    g = load_file(os.path.join(HERE, 'golden', 'golden_vfe.safetensors'))
    vit = O.VFE_VIT
    fe, sd, proj = make_vfe(vit)
    assert fe.input_dim == 512
    hu = W.make_hu(2, vit, seed=31)
    feats = fe(hu.cuda())
    torch.cuda.synchronize()
    assert feats.shape == (2, 512) and feats.dtype == torch.float32
    # the reference's f32 [-1, 1] input takes the int16 path bit-for-bit
    assert torch.equal(fe(O.normalize_hu(hu)), feats)
    e = rel(feats, g['out.features'])
    print(f'VFE features vs reference fixture: rel err {e:.3e}, max abs '
          f'{(feats.cpu() - g["out.features"]).abs().max().item():.3e}')
    assert e < 1e-2
    # stages: the same spatial stack the extractor runs, via the encoder's own pieces
    from ctclip_mi355x import functional as Fn
    ve = fe.vision_encoder
    x = hu.cuda()
    pe = ve.to_patch_emb
    with torch.no_grad():
        xf, xb = Fn.PatchEmbedFn.apply(x, pe[1].weight, pe[1].bias, pe[2].weight, pe[2].bias, pe[3].weight,
                                       pe[3].bias, ve.temporal_patch_size, ve.patch_size[0], True,
                                       ve._offsets(x.shape, x.device))
        yf, _ = ve.enc_spatial_transformer.run(xf, xb, Fn.Geo(2, 4, 8, 8, ve.heads, ve.dim_head, 0), None)
    assert rel(xf, g['out.patch_emb'].reshape(-1, 512)) < 1e-2
    assert rel(yf, g['out.spatial_out'].reshape(-1, 512)) < 2e-2
    assert rel(yf.view(2, -1, 512).mean(1), g['out.pooled']) < 2e-2


def test_vfe_position_bias_variant():
    vit = O.VFE_VIT
    fe, sd, proj = make_vfe(vit, position_bias=True)
    hu = W.make_hu(2, vit, seed=32)
    feats = fe(hu.cuda())
    with torch.no_grad():
        ref = O.vision_features(sd, 'visual_transformer.', O.normalize_hu(hu), vit, proj, position_bias=True)
    e = rel(feats, ref)
    print(f'VFE (CPB bias) vs oracle: rel err {e:.3e}')
    assert e < 1e-2


def test_vfe_full_size():
    """configs[4]'s volume: (1, 1, 240, 480, 480) int16 -> (1, 512)."""
    vit = O.ViTConfig()
    fe, sd, proj = make_vfe(vit)
    hu = W.make_hu(1, vit, seed=33)
    feats = fe(hu.cuda())
    torch.cuda.synchronize()
    assert feats.shape == (1, 512)
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    with torch.no_grad():
        ref = O.vision_features(sd, 'visual_transformer.', O.normalize_hu(hu), vit, proj)
    e = rel(feats, ref)
    print(f'VFE full size vs oracle: rel err {e:.3e}')
    assert e < 1e-2
    with pytest.raises(ValueError):
        fe(torch.zeros(1, 1, 240, 400, 400, dtype=torch.int16))
