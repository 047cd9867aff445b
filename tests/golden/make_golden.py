"""Generate golden fixtures by running the REFERENCE's own ct_clip modules on CPU.

Run in the build container only (needs /root/reference, read-only):
    python tests/golden/make_golden.py [--base]

What it does: imports transformers first, installs import-time stubs for
deps missing offline (beartype -> no-op decorator; torchvision -> import-only names;
vector_quantize_pytorch -> the cosine-VQ restatement of oracle/ctclip_oracle.vq_forward,
since the pinned 1.1.2 package is absent), maps the reference's hard-coded
torch.device('cuda') to CPU, builds CTViT(use_vgg_and_gan=False) + a locally initialised
BertModel + CTCLIP, loads the name-seeded recipe weights (oracle/weights.py) with
strict=True, and records inputs / per-stage outputs / loss / grads as safetensors.

The fixtures are DATA (inputs + expected outputs); nothing from the reference's source is
copied into them.
"""
from __future__ import annotations

import argparse
import os
import sys
import types

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = '/root/reference/CTPA_CLIP'
sys.path.insert(0, REPO)

import transformers  # noqa: E402  (must import before the torchvision stub)
from transformers import BertModel, BertConfig as HFBertConfig  # noqa: E402
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from safetensors.torch import save_file  # noqa: E402

from oracle import ctclip_oracle as O  # noqa: E402
from oracle import weights as W  # noqa: E402


def install_stubs():
    bt = types.ModuleType('beartype')
    bt.beartype = lambda f: f
    sys.modules['beartype'] = bt
    tv = types.ModuleType('torchvision')
    tvt = types.ModuleType('torchvision.transforms')

    class _T:
        def __init__(self, *a, **k):
            pass

        def __call__(self, x):
            return x
    for n in ['Compose', 'Resize', 'ToTensor', 'ColorJitter', 'RandomGrayscale', 'RandomHorizontalFlip',
              'GaussianBlur', 'RandomResizedCrop', 'Normalize']:
        setattr(tvt, n, _T)
    tvm = types.ModuleType('torchvision.models')
    tvu = types.ModuleType('torchvision.utils')
    tv.transforms, tv.models, tv.utils = tvt, tvm, tvu
    sys.modules.update({'torchvision': tv, 'torchvision.transforms': tvt,
                        'torchvision.models': tvm, 'torchvision.utils': tvu})

    vqm = types.ModuleType('vector_quantize_pytorch')

    class _Codebook(nn.Module):
        def __init__(self, dim, codebook_size):
            super().__init__()
            self.register_buffer('initted', torch.ones(1))
            self.register_buffer('cluster_size', torch.zeros(1, codebook_size))
            self.register_buffer('embed', torch.zeros(1, codebook_size, dim))

    class VectorQuantize(nn.Module):
        def __init__(self, dim, codebook_size, use_cosine_sim=False, decay=0.8, **kw):
            super().__init__()
            assert use_cosine_sim
            self.decay = decay
            self._codebook = _Codebook(dim, codebook_size)

        @property
        def codebook(self):
            return self._codebook.embed[0]

        def forward(self, x, mask=None):
            cb = self._codebook
            q, ind, ne, ncs = O.vq_forward(x, cb.embed, cb.cluster_size, self.training, self.decay)
            if self.training:
                cb.embed.copy_(ne)
                cb.cluster_size.copy_(ncs)
            return q, ind, torch.zeros(1)
    vqm.VectorQuantize = VectorQuantize
    sys.modules['vector_quantize_pytorch'] = vqm


class _TorchProxy:
    """Delegates to torch but maps torch.device(...) to CPU (the reference hard-codes cuda
    at ctvit.py:61,110,274,316,356,398 and attention.py:135,171,195,219,260)."""

    def __getattr__(self, n):
        return getattr(torch, n)

    @staticmethod
    def device(*a, **k):
        return torch.device('cpu')


def import_reference():
    install_stubs()
    sys.path.insert(0, REF)
    import ct_clip.attention as A
    import ct_clip.ctvit as V
    import ct_clip.ct_clip as C
    A.torch = _TorchProxy()
    V.torch = _TorchProxy()

    class _Tok:
        @staticmethod
        def from_pretrained(*a, **k):
            return None
    C.BertTokenizer = _Tok
    return A, V, C


def build_reference(cfg: O.ClipConfig, V, C):
    vc = cfg.vit
    vit = V.CTViT(dim=vc.dim, codebook_size=vc.codebook_size, image_size=vc.image_size,
                  patch_size=vc.patch_size, temporal_patch_size=vc.temporal_patch_size,
                  spatial_depth=vc.spatial_depth, temporal_depth=vc.temporal_depth,
                  dim_head=vc.dim_head, heads=vc.heads, use_vgg_and_gan=False)
    bc = cfg.bert
    bert = BertModel(HFBertConfig(vocab_size=bc.vocab_size, hidden_size=bc.hidden,
                                  num_hidden_layers=bc.layers, num_attention_heads=bc.heads,
                                  intermediate_size=bc.intermediate,
                                  max_position_embeddings=bc.max_position, type_vocab_size=bc.type_vocab,
                                  hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0,
                                  attn_implementation='eager'))
    clip = C.CTCLIP(image_encoder=vit, text_encoder=bert, dim_text=bc.hidden, dim_image=cfg.dim_image,
                    dim_latent=cfg.dim_latent, extra_latent_projection=False, use_mlm=False,
                    downsample_image_embeds=False, use_all_token_embeds=False)
    return clip


class _Text:
    def __init__(self, ids, mask):
        self.input_ids = ids
        self.attention_mask = mask


def run(cfg, batch, text_len, ragged, with_grads, tag, V, C, save_full_state):
    clip = build_reference(cfg, V, C)
    sd = W.make_state_dict(cfg)
    ref_keys = set(clip.state_dict().keys())
    assert ref_keys == set(sd.keys()), (sorted(ref_keys ^ set(sd.keys())))[:20]
    clip.load_state_dict(sd, strict=True)
    for p in clip.parameters():          # fine_tuning_ctclip.py:6-14
        p.requires_grad = False
    for p in clip.visual_transformer.parameters():
        p.requires_grad = True
    for p in clip.text_transformer.parameters():
        p.requires_grad = True

    hu = W.make_hu(batch, cfg.vit)
    video = O.normalize_hu(hu)
    ids, mask = W.make_text(batch, text_len, cfg.bert.vocab_size, ragged=ragged)

    cap = {}
    vt = clip.visual_transformer
    hooks = [
        vt.to_patch_emb.register_forward_hook(lambda m, i, o: cap.__setitem__('patch_emb', o.detach().clone())),
        vt.spatial_rel_pos_bias.register_forward_hook(lambda m, i, o: cap.__setitem__('cpb', o.detach().clone())),
        vt.enc_spatial_transformer.register_forward_hook(
            lambda m, i, o: cap.__setitem__('spatial_out', o.detach().clone())),
        vt.enc_temporal_transformer.register_forward_hook(
            lambda m, i, o: cap.__setitem__('temporal_out', o.detach().clone())),
        vt.vq.register_forward_hook(lambda m, i, o: cap.__setitem__('vq_indices', o[1].detach().clone())),
        clip.to_text_latent.register_forward_hook(lambda m, i, o: cap.__setitem__('text_proj', o.detach().clone())),
        clip.to_visual_latent.register_forward_hook(
            lambda m, i, o: cap.__setitem__('image_proj', o.detach().clone())),
        clip.text_transformer.register_forward_hook(
            lambda m, i, o: cap.__setitem__('enc_text', o[0].detach().clone())),
    ]
    clip.train()
    loss = clip(_Text(ids, mask), video, device='cpu', return_loss=True)
    out = {'in.hu': hu, 'in.ids': ids, 'in.mask': mask, 'out.loss': loss.detach().reshape(1)}
    for k, v in cap.items():
        out['out.' + k] = v
    out['out.new_embed'] = vt.vq._codebook.embed.detach().clone()
    out['out.new_cluster_size'] = vt.vq._codebook.cluster_size.detach().clone()
    if with_grads:
        loss.backward()
        for n, p in clip.named_parameters():
            if p.grad is not None:
                out['grad.' + n] = p.grad.detach().clone()
    for h in hooks:
        h.remove()
    # eval branch: zero-shot scores (ct_clip.py:805-807); codebook restored first
    clip.load_state_dict(sd, strict=True)
    clip.eval()
    with torch.no_grad():
        out['out.eval_scores'] = clip(_Text(ids, mask), video, device='cpu', return_loss=False).detach()
    if save_full_state:
        for k, v in sd.items():
            out['sd.' + k] = v
    out = {k: v.contiguous() for k, v in out.items()}
    path = os.path.join(HERE, f'golden_{tag}.safetensors')
    save_file(out, path, metadata={'batch': str(batch), 'text_len': str(text_len), 'ragged': str(ragged),
                                   'generator': 'tests/golden/make_golden.py',
                                   'reference': 'sharonct/CTPA-CLIP @ 2025-06-20 (ct_clip/*.py)'})
    print(tag, 'loss', float(loss.detach()), 'keys', len(out), '->', path)


def shrink_base(out_keys_keep=None):
    pass


def run_zero_shot(V, C):
    """Zero-shot fixture (tiny config): the reference's own eval loop of
    ct_clip/ctclip_inference.py:305-315 -- per volume (batch 1) and per pathology, CTCLIP.forward on
    the 2-prompt pair, softmax over the pair, keep entry 0.  Prompt ids are synthetic (the
    CXR-BERT tokenizer is not available offline): rows (2j, 2j+1) = pathology j's pair."""
    cfg = O.TINY
    clip = build_reference(cfg, V, C)
    sd = W.make_state_dict(cfg)
    clip.load_state_dict(sd, strict=True)
    clip.eval()
    n, P = 2, 3
    hu = W.make_hu(n, cfg.vit, seed=77)
    video = O.normalize_hu(hu)
    ids, mask = W.make_text(2 * P, 16, cfg.bert.vocab_size, seed=99, ragged=True)
    probs, scores = torch.empty(n, P), torch.empty(n, P, 2)
    with torch.no_grad():
        for v in range(n):
            for j in range(P):
                s = clip(_Text(ids[2 * j:2 * j + 2], mask[2 * j:2 * j + 2]), video[v:v + 1], device='cpu')
                scores[v, j] = s
                probs[v, j] = torch.nn.Softmax(dim=0)(s)[0]
    out = {'in.hu': hu, 'in.ids': ids, 'in.mask': mask, 'out.probs': probs, 'out.scores': scores}
    path = os.path.join(HERE, 'golden_zeroshot_tiny.safetensors')
    save_file({k: v.contiguous() for k, v in out.items()}, path,
              metadata={'generator': 'tests/golden/make_golden.py --zero-shot',
                        'reference': 'sharonct/CTPA-CLIP @ 2025-06-20 (ct_clip/ctclip_inference.py:305-315)'})
    print('zero-shot probs', probs.tolist(), '->', path)


def run_recon(V, C):
    """Reconstruction fixture (tiny config): the reference CTViT built with
    use_vgg_and_gan=False, forward(video, return_recons=True) in train mode (ct_clip/ctvit.py:
    377-451: encode -> VQ -> decode -> MSE), its loss / recon / VQ indices and parameter grads."""
    cfg = O.TINY
    clip = build_reference(cfg, V, C)
    sd = W.make_state_dict(cfg)
    clip.load_state_dict(sd, strict=True)
    vit = clip.visual_transformer
    vit.train()
    cap = {}
    vit.vq.register_forward_hook(lambda m, i, o: cap.__setitem__('vq_indices', o[1].detach().clone()))
    hu = W.make_hu(2, cfg.vit, seed=55)
    video = O.normalize_hu(hu)
    loss, recon = vit(video, return_recons=True)
    loss.backward()
    out = {'in.hu': hu, 'out.loss': loss.detach().reshape(1), 'out.recon': recon.detach(),
           'out.vq_indices': cap['vq_indices']}
    for n, prm in vit.named_parameters():
        if prm.grad is not None:
            out['grad.visual_transformer.' + n] = prm.grad.detach().clone()
    path = os.path.join(HERE, 'golden_recon_tiny.safetensors')
    save_file({k: v.contiguous() for k, v in out.items()}, path,
              metadata={'generator': 'tests/golden/make_golden.py --recon',
                        'reference': 'sharonct/CTPA-CLIP @ 2025-06-20 (ct_clip/ctvit.py:333-451)'})
    print('recon loss', float(loss), 'grads', sum(k.startswith('grad.') for k in out), '->', path)


def run_vfe(V, C):
    """VisionFeatureExtractor fixture (configs[4], ctpa_report/vqa_meditron.py:26-131): base widths
    on a reduced volume (160 x 160 x 40 -> 4 x 8 x 8 tokens, 4 spatial layers).  The reference's own
    modules run the extractor's forward (:91-123) with the one repair it needs -- video_shape for
    the spatial transformer, whose absence makes PEG raise and the forward return torch.randn --
    and no attn_bias, as its call has none.  vqa_meditron.py itself cannot be imported offline (it
    loads the CT-CLIP_v2.pt checkpoint at import through ct_clip.pretrained_model and needs peft),
    so its projector -- nn.Sequential(Linear, LayerNorm, GELU) (:42-46) -- is built here as torch
    modules with the oracle/weights.make_projector recipe."""
    vit_cfg = O.VFE_VIT
    cfg = O.ClipConfig(vit=vit_cfg, bert=O.TINY.bert, dim_latent=512)
    clip = build_reference(cfg, V, C)
    sd = W.make_state_dict(cfg)
    clip.load_state_dict(sd, strict=True)
    vt = clip.visual_transformer
    vt.eval()
    proj = W.make_projector(512, 512)
    fp = nn.Sequential(nn.Linear(512, 512), nn.LayerNorm(512), nn.GELU())
    fp.load_state_dict({k[len('feature_projector.'):]: v for k, v in proj.items()}, strict=True)
    hu = W.make_hu(2, vit_cfg, seed=31)
    x = O.normalize_hu(hu)
    with torch.no_grad():
        pe = vt.to_patch_emb(x)                                    # vqa_meditron.py:101
        b, t, h, w, d = pe.shape
        si = pe.reshape(-1, h * w, d)                              # its local rearrange, :134-141
        sf = vt.enc_spatial_transformer(si, video_shape=(b, t, h, w))   # :107 + video_shape
        pooled = F.adaptive_avg_pool3d(sf.reshape(b, t, h, w, d).permute(0, 4, 1, 2, 3), (1, 1, 1)).reshape(b, d)
        feats = fp(pooled)                                         # :120
    # input: W.make_hu(2, vit, seed=31), regenerated by the tests
    out = {'out.patch_emb': pe, 'out.spatial_out': sf.reshape(b, t, h, w, d), 'out.pooled': pooled,
           'out.features': feats}
    path = os.path.join(HERE, 'golden_vfe.safetensors')
    save_file({k: v.contiguous() for k, v in out.items()}, path,
              metadata={'generator': 'tests/golden/make_golden.py --vfe',
                        'reference': 'sharonct/CTPA-CLIP @ 2025-06-20 (ctpa_report/vqa_meditron.py:91-123, '
                                     'ct_clip/ctvit.py:169-174, ct_clip/attention.py:280-333)'})
    print('vfe features', feats.shape, float(feats.abs().mean()), '->', path)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--base', action='store_true', help='also write the base-config B=2 fixture')
    ap.add_argument('--zero-shot', action='store_true', help='only write the zero-shot fixture')
    ap.add_argument('--recon', action='store_true', help='only write the reconstruction fixture')
    ap.add_argument('--vfe', action='store_true', help='only write the VisionFeatureExtractor fixture')
    args = ap.parse_args()
    torch.set_num_threads(os.cpu_count())
    A, V, C = import_reference()
    if args.vfe:
        run_vfe(V, C)
        return
    if args.zero_shot:
        run_zero_shot(V, C)
        return
    if args.recon:
        run_recon(V, C)
        return
    run(O.TINY, batch=4, text_len=16, ragged=True, with_grads=True, tag='tiny', V=V, C=C,
        save_full_state=False)
    if args.base:
        run_base(V, C)


def run_base(V, C):
    """Base config, B=2, 128-token text: store only compact outputs (indices, latents,
    loss, samples) — the weights come from the recipe on both sides."""
    cfg = O.BASE
    clip = build_reference(cfg, V, C)
    sd = W.make_state_dict(cfg)
    clip.load_state_dict(sd, strict=True)
    hu = W.make_hu(2, cfg.vit)
    video = O.normalize_hu(hu)
    ids, mask = W.make_text(2, 128, cfg.bert.vocab_size)
    cap = {}
    vt = clip.visual_transformer
    vt.to_patch_emb.register_forward_hook(lambda m, i, o: cap.__setitem__('patch_emb', o.detach()))
    vt.spatial_rel_pos_bias.register_forward_hook(lambda m, i, o: cap.__setitem__('cpb', o.detach()))
    vt.enc_spatial_transformer.register_forward_hook(lambda m, i, o: cap.__setitem__('spatial_out', o.detach()))
    vt.enc_temporal_transformer.register_forward_hook(lambda m, i, o: cap.__setitem__('temporal_out', o.detach()))
    vt.vq.register_forward_hook(lambda m, i, o: cap.__setitem__('vq_indices', o[1].detach()))
    clip.text_transformer.register_forward_hook(lambda m, i, o: cap.__setitem__('enc_text', o[0].detach()))
    for p in clip.parameters():
        p.requires_grad = False
    clip.train()
    with torch.no_grad():
        loss = clip(_Text(ids, mask), video, device='cpu', return_loss=True)
        t_lat, i_lat, _ = None, None, None
    # latents via the oracle-independent path: re-run eval latents on the reference
    clip.load_state_dict(sd, strict=True)
    clip.eval()
    with torch.no_grad():
        t_lat, i_lat, enc = clip(_Text(ids, mask), video, device='cpu', return_latents=True)
    out = {
        'out.loss': loss.reshape(1),
        'out.text_latents': t_lat, 'out.image_latents': i_lat,
        'out.vq_indices': cap['vq_indices'].to(torch.int32),
        'out.cpb_rows': cap['cpb'][:, :4, :].contiguous(),
        'out.patch_emb_head': cap['patch_emb'].reshape(-1, cfg.vit.dim)[:256].contiguous(),
        'out.spatial_out_head': cap['spatial_out'].reshape(-1, cfg.vit.dim)[:256].contiguous(),
        'out.temporal_out_head': cap['temporal_out'].reshape(-1, cfg.vit.dim)[:256].contiguous(),
        'out.enc_text_cls': cap['enc_text'][:, 0, :].contiguous(),
        'out.patch_emb_sum': cap['patch_emb'].double().reshape(2, -1, cfg.vit.dim).sum(1).float(),
        'out.temporal_out_sum': cap['temporal_out'].double().reshape(2, -1, cfg.vit.dim).sum(1).float(),
    }
    path = os.path.join(HERE, 'golden_base_b2.safetensors')
    save_file({k: v.contiguous() for k, v in out.items()}, path,
              metadata={'batch': '2', 'text_len': '128', 'generator': 'tests/golden/make_golden.py --base'})
    print('base loss', float(loss), '->', path)


if __name__ == '__main__':
    main()
