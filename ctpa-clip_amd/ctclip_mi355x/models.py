"""Constructors mirroring ct_clip/pretrained_model.py:17-42 (CTViT + BERT-base + CTCLIP)."""
from __future__ import annotations

from .bert import BertConfig, BertModel
from .ct_clip import CTCLIP
from .ctvit import CTViT

BASE_VIT = dict(dim=512, codebook_size=8192, image_size=480, patch_size=20, temporal_patch_size=10,
                spatial_depth=4, temporal_depth=4, dim_head=32, heads=8)


def build_ctclip(vit=None, bert=None, dim_latent=512, frames=240):
    """CT-CLIP as the reference assembles it.  ``vit`` = CTViT kwargs (default: base),
    ``bert`` = BertConfig (default: BERT-base as CXR-BERT-specialized).  The flattened image
    embedding width follows from the ViT grid: (image/patch)^2 * dim (ct_clip.py:724,740)."""
    vk = dict(BASE_VIT)
    vk.update(vit or {})
    image_encoder = CTViT(**vk, use_vgg_and_gan=False)
    text_encoder = BertModel(bert or BertConfig())
    grid = vk['image_size'] // vk['patch_size']
    dim_image = grid * grid * vk['dim']
    return CTCLIP(image_encoder=image_encoder, text_encoder=text_encoder,
                  dim_text=text_encoder.config.hidden_size, dim_image=dim_image, dim_latent=dim_latent,
                  extra_latent_projection=False, use_mlm=False, downsample_image_embeds=False,
                  use_all_token_embeds=False)


def set_finetune_trainable(model):
    """ct_clip/fine_tuning_ctclip.py:6-14: freeze all, unfreeze the visual and text transformers."""
    for p in model.parameters():
        p.requires_grad = False
    for p in model.visual_transformer.parameters():
        p.requires_grad = True
    for p in model.text_transformer.parameters():
        p.requires_grad = True
    # parameters that exist in the reference's state_dict but never receive a gradient on the
    # contrastive path (ct_clip/ctvit.py:162-167,189-197; attention.py:114,117): keep them out of
    # the optimiser arena, exactly as DDP(find_unused_parameters=True) would skip them.
    vt = model.visual_transformer
    for mod in (vt.to_patch_emb_first_frame, vt.to_pixels_first_frame, vt.to_pixels):
        for p in mod.parameters():
            p.requires_grad = False
    for tr in (vt.enc_spatial_transformer, vt.enc_temporal_transformer):
        for _, attn, _, _ in tr.layers:
            attn.null_kv.requires_grad = False
            attn.context_norm.gamma.requires_grad = False
    for p in model.text_transformer.pooler.parameters():
        p.requires_grad = False
    return model
