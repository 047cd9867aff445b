"""CPU checks of the drop-in boundary: the product model's state_dict layout equals the
reference's (as pinned by the golden generator, which asserts the recipe keys == the reference
CTCLIP.state_dict() keys), and the C-ABI library exports every symbol include/ctclip_hip.h declares."""
import ctypes
import os
import re

import pytest
import torch

from oracle import ctclip_oracle as O
from oracle import weights as W

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _small_cfg():
    vit = O.ViTConfig(dim=512, codebook_size=512, image_size=80, patch_size=20, temporal_patch_size=10,
                      spatial_depth=1, temporal_depth=1, dim_head=32, heads=8, frames=20)
    bert = O.BertConfig(vocab_size=500, hidden=256, layers=1, heads=4, intermediate=512, max_position=64)
    return O.ClipConfig(vit=vit, bert=bert, dim_latent=64)


def _product(cfg):
    from ctclip_mi355x.models import build_ctclip
    from ctclip_mi355x.bert import BertConfig
    v = cfg.vit
    vit = dict(dim=v.dim, codebook_size=v.codebook_size, image_size=v.image_size, patch_size=v.patch_size,
               temporal_patch_size=v.temporal_patch_size, spatial_depth=v.spatial_depth,
               temporal_depth=v.temporal_depth, dim_head=v.dim_head, heads=v.heads)
    b = cfg.bert
    bert = BertConfig(vocab_size=b.vocab_size, hidden_size=b.hidden, num_hidden_layers=b.layers,
                      num_attention_heads=b.heads, intermediate_size=b.intermediate,
                      max_position_embeddings=b.max_position)
    return build_ctclip(vit, bert, cfg.dim_latent)


def test_state_dict_layout_matches_reference():
    cfg = _small_cfg()
    model = _product(cfg)
    ours = {k: tuple(v.shape) for k, v in model.state_dict().items()}
    ref = {k: tuple(shape) for k, (_, shape) in W.clip_keys(cfg).items()}
    assert set(ours) == set(ref), sorted(set(ours) ^ set(ref))[:20]
    assert all(ours[k] == ref[k] for k in ref)
    sd = W.make_state_dict(cfg)
    missing, unexpected = model.load_state_dict(sd, strict=True), None
    assert model.visual_transformer.vq.codebook.shape == (512, 512)


def test_finetune_trainable_set():
    from ctclip_mi355x.models import set_finetune_trainable
    model = set_finetune_trainable(_product(_small_cfg()))
    names = [n for n, p in model.named_parameters() if p.requires_grad]
    assert all(n.startswith(('visual_transformer.', 'text_transformer.')) for n in names)
    assert not model.to_visual_latent.weight.requires_grad and not model.temperature.requires_grad


def test_cabi_exports_every_declared_symbol():
    hdr = open(os.path.join(REPO, 'include', 'ctclip_hip.h')).read()
    names = sorted(set(re.findall(r'\bint\s+(ctclip_\w+)\s*\(', hdr)))
    assert len(names) > 30
    from ctclip_mi355x import _lib
    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    # every declared symbol has a ctypes signature on the Python side
    assert not [n for n in names if n not in _lib._SIGS]
    assert lib.ctclip_version() == 2


def test_product_has_no_cpu_fallback():
    """The product package never imports the oracle and raises without a GPU."""
    pkg = os.path.join(REPO, 'ctpa-clip_amd', 'ctclip_mi355x')
    for f in os.listdir(pkg):
        if f.endswith('.py'):
            src = open(os.path.join(pkg, f)).read()
            assert 'oracle' not in src.replace('oracle/ctclip_oracle', ''), f
