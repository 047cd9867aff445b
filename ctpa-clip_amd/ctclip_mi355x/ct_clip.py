"""CTCLIP (ct_clip/ct_clip.py:407-901) — drop-in constructor / forward signature and state_dict
layout, with the image tower, text tower, projections and InfoNCE running on HIP kernels.

Supported configuration = the one the reference trains (pretrained_model.py:31-42):
external image / text encoders, use_mlm=False, use_visual_ssl=False, use_all_token_embeds=False,
downsample_image_embeds=False, no multiview augmentation.  Anything else raises.
"""
from __future__ import annotations

import copy
import os
from pathlib import Path

import torch
from torch import nn

from . import dist_sync
from . import functional as Fn
from . import streams


# queue BERT's forward before the image tower's (A/B switch, default: image tower first)
TEXT_FWD_FIRST = os.environ.get('CTCLIP_TEXT_FWD_FIRST', '0') != '0'
# BERT's forward (text stream) starts after the image tower's patch embedding instead of with it: the
# patch LayerNorm is HBM-bound (0.43 ms alone, ~1.1 ms beside BERT's first kernels in round 4) and BERT
# is hidden behind the 3D-ViT either way.  CTCLIP_TEXT_GATE=0: start together (A/B).
TEXT_GATE = os.environ.get('CTCLIP_TEXT_GATE', '1') != '0'
# where the training VQ's codebook EMA update is queued on the auxiliary stream (A/B): '0' right
# after the VQ (its ~0.34 ms of short workgroups then hold the CUs the projection's slab reduction
# waits for: 5 -> 321 us in step, r05f_seq.txt), '1' after the image projection (the loss kernel and
# the backward's first launches wait instead), '2' (default) after the optimizer step, beside the
# next step's forward -- only when CTClipTrainer owns the step (train_step sets ema_after_step,
# optimizer_step calls flush_ema; any codebook reader, the next VQ or state_dict, queues a pending
# update first); a plain model(...) call in train mode gets site '1', so the codebook read after it
# is the updated one, as the reference updates it inside forward.  Measured (r05m_ema_site_ab.log):
# '2' 204.30 vs '1' 203.70 pairs/s; '1' vs '0' within noise (r05g_ema_ab_env.log).  '3' (round 6): as
# '2', but the trainer leaves the update pending and the NEXT step's image tower queues it once its
# patch embedding is queued (ctvit.encode_tokens), so it runs beside the GEMM-bound first layer
# instead of beside the HBM-bound patch LayerNorm (any codebook reader still queues it first)
DEFER_EMA = os.environ.get('CTCLIP_DEFER_EMA', '2')


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


def l2norm(t):
    return nn.functional.normalize(t, dim=-1)


class CTCLIP(nn.Module):
    def __init__(self, *, image_encoder=None, text_encoder=None, dim_text=512, dim_image=512, dim_latent=512,
                 num_text_tokens=28897, text_enc_depth=6, text_seq_len=256, text_heads=8, text_dim_head=64,
                 text_has_cls_token=False, text_pad_id=0, text_rotary_pos_emb=False, text_causal_mask=False,
                 text_eos_id=None, text_encode_without_mask=False, visual_enc_depth=6, visual_heads=8,
                 visual_dim_head=64, visual_image_size=256, visual_patch_size=32, visual_patch_dropout=0.5,
                 visual_has_cls_token=False, channels=3, use_all_token_embeds=False, downsample_image_embeds=False,
                 decoupled_contrastive_learning=False, extra_latent_projection=False, use_mlm=False,
                 text_ssl_loss_weight=0.05, use_visual_ssl=False, visual_ssl=None, visual_ssl_type='simsiam',
                 visual_ssl_hidden_layer=-1, simclr_temperature=0.1, image_ssl_loss_weight=0.05,
                 multiview_loss_weight=0.1, checkpoint_during_training=False, **kwargs):
        super().__init__()
        unsupported = dict(use_all_token_embeds=use_all_token_embeds, downsample_image_embeds=downsample_image_embeds,
                           decoupled_contrastive_learning=decoupled_contrastive_learning, use_mlm=use_mlm,
                           use_visual_ssl=use_visual_ssl or visual_ssl is not None,
                           text_causal_mask=text_causal_mask)
        bad = [k for k, v in unsupported.items() if v]
        if bad:
            raise NotImplementedError(f'CTCLIP options outside the contrastive hot path: {bad}')
        if image_encoder is None or text_encoder is None:
            raise NotImplementedError('the built-in VisionTransformer / TextTransformer are never used by the '
                                      'reference (pretrained_model.py:31-42); pass image_encoder and text_encoder')
        self.dim_text = dim_text
        self.dim_image = dim_image
        self.dim_latent = dim_latent
        self.text_transformer = text_encoder
        self.visual_transformer = image_encoder
        self.to_text_latent = nn.Linear(dim_text, dim_latent, bias=False)
        self.to_visual_latent = nn.Linear(dim_image, dim_latent, bias=False)
        self.temperature = nn.Parameter(torch.tensor(1.))
        self.extra_latent_projection = extra_latent_projection
        self.to_text_latent_extra = copy.deepcopy(self.to_text_latent)
        self.to_visual_latent_extra = copy.deepcopy(self.to_visual_latent)
        self.multiview_loss_weight = multiview_loss_weight
        self._wvis = (None, None)
        self.defer_text_backward = False     # set by CTClipTrainer (see encode)
        self._deferred_text = None
        self._deferred_image = None
        self._t_gather = None
        self.ema_after_step = False          # set by CTClipTrainer.train_step (DEFER_EMA '2')

    # ------------------------------------------------------------------ checkpoint
    def load(self, path):
        """``CTCLIP.load`` (ct_clip/ct_clip.py:593-597): strict=False; weights-only safe loader."""
        path = Path(path)
        assert path.exists()
        pt = torch.load(str(path), map_location='cpu', weights_only=True)
        return self.load_state_dict(pt, strict=False)

    def state_dict(self, *args, **kwargs):
        """The reference key layout; a text-tower Adam the trainer deferred to the next step
        (CTClipTrainer(defer_text_adam=True)) is queued first, and the caller's stream is ordered
        after the text stream (BERT's Adam) and the auxiliary stream (the codebook EMA), so the
        tensors returned -- and any copy of them queued on the current stream, e.g. torch.save --
        hold the updated weights."""
        if self._vq_state() is not None:
            self._vq_state().flush_ema()
        for p in self.text_transformer.parameters():
            if p.is_cuda:
                streams.flush_text(p.device)
                streams.join_text(p.device)
                streams.join_aux(p.device)
            break
        return super().state_dict(*args, **kwargs)

    # ------------------------------------------------------------------ helpers
    def _vq_state(self):
        """The image tower's VQ cache (functional.VQState), or None for another image encoder."""
        return getattr(getattr(self.visual_transformer, 'vq', None), 'state', None)

    def flush_ema(self):
        """Queue a deferred codebook EMA update now (auxiliary stream; see DEFER_EMA)."""
        vqs = self._vq_state()
        if vqs is not None:
            vqs.flush_ema()

    def _visual_weight_bf16(self, W):
        """bf16 to_visual_latent weight (151 M parameters): the Adam-kept shadow when W trains,
        else a cast cached until W changes.  Frozen in the fine-tune configuration
        (fine_tuning_ctclip.py:6-14), so it is cast once, not every step (0.23 ms per recast)."""
        from . import kernels as K
        from . import functional as Fn
        sh = Fn.shadow_bf16(W)
        if sh is not None:
            return sh
        # only an optimizer arena member is written behind torch's version counter (raw pointers)
        in_arena = getattr(W, '_ctclip_flat', None) is not None
        key = (W.data_ptr(), W._version, K.weights_epoch() if in_arena else -1)
        if self._wvis[0] != key:
            self._wvis = (key, K.cast_bf16(W.detach().contiguous()))
        return self._wvis[1]

    def _project(self, W, Wb, pooled, pooled_b):
        # (in the f32 image-tower mode ImageProjFn's forward is the exact-f32 product, precise.py)
        return Fn.ImageProjFn.apply(pooled, pooled_b, W, Wb)

    def encode(self, text, image, gather=False):
        """Text + image towers and raw latents: (enc_text (B,L,768), pooled (B, h*w*d),
        text_raw (B, dl), image_raw (B, dl)).  ``gather``: the caller will compute the global-batch
        loss, so under torch.distributed the text latents' all-gather starts here (every rank makes
        the same call); other callers (scores, encodings) issue no collective."""
        # The host queues the image tower first (its ~16 ms of GPU work keep this stream busy while
        # the host queues BERT's many small launches), BERT on the text stream (streams.py) ordered
        # only after an event taken before the image tower, so the two run side by side.
        dev = image.device
        ready = torch.cuda.current_stream(dev).record_event() if streams.text_stream(dev) else None
        if TEXT_FWD_FIRST:      # A/B: BERT's launches queued before the image tower's
            enc_text = self.text_transformer(text.input_ids, attention_mask=text.attention_mask, join=False,
                                             ready=ready)[0]
            pooled, pooled_b = self.visual_transformer.encode_pooled(image)
        else:
            vqs = self._vq_state()
            if vqs is not None:
                vqs.defer_ema = DEFER_EMA != '0' and self.visual_transformer.training
            try:
                pooled, pooled_b = self.visual_transformer.encode_pooled(image)
            finally:
                if vqs is not None:
                    vqs.defer_ema = False
            gate = getattr(self.visual_transformer, '_patch_done', None)
            if TEXT_GATE and ready is not None and gate is not None:
                ready = gate
            enc_text = self.text_transformer(text.input_ids, attention_mask=text.attention_mask, join=False,
                                             ready=ready)[0]
        ts = streams.text_stream(dev)
        with torch.cuda.stream(ts) if ts is not None else _nullctx():
            t_raw = Fn.TextProjFn.apply(enc_text[:, 0, :].contiguous(), self.to_text_latent.weight)
            # N > 1: the text latents' all-gather goes out from the text stream now, beside the
            # 3D-ViT forward still running on the main stream (SURVEY 8(e) overlap)
            self._t_gather = dist_sync.start_gather(t_raw) if gather and dist_sync.world_rank()[0] > 1 else None
        streams.join_text(dev)
        if ts is not None:
            t_raw.record_stream(torch.cuda.current_stream(dev))
        if self.defer_text_backward and torch.is_grad_enabled() and t_raw.requires_grad:
            # the trainer back-propagates the text tower AFTER the loss / 3D-ViT graph
            # (CTClipTrainer.forward_backward): the long ViT chain is queued first, and BERT's
            # backward, queued while the GPU still works through it, runs beside it on the text
            # stream -- ordered only after an event taken when the loss produced its gradient
            leaf = t_raw.detach().requires_grad_(True)
            d = self._deferred_text = [t_raw, leaf, None]
            if ts is not None:
                def mark(g):
                    d[2] = torch.cuda.current_stream(dev).record_event()
                leaf.register_hook(mark)
            t_raw = leaf
        W = self.to_visual_latent.weight
        i_raw = self._project(W, self._visual_weight_bf16(W), pooled, pooled_b)
        if DEFER_EMA == '1' or (DEFER_EMA in ('2', '3') and not self.ema_after_step):
            self.flush_ema()               # the codebook EMA, after the projection
        if self.defer_text_backward and torch.is_grad_enabled() and i_raw.requires_grad:
            # the image tower's backward is deferred too (CTClipTrainer.forward_backward): BERT's
            # backward -- and its gradient buckets' all-reduces -- are queued before the 3D-ViT's
            ileaf = i_raw.detach().requires_grad_(True)
            self._deferred_image = [i_raw, ileaf]
            i_raw = ileaf
        return enc_text, pooled, t_raw, i_raw

    def forward(self, text, image, device=None, return_loss=False, return_encodings=False, return_latents=False,
                freeze_image_encoder=False, freeze_text_encoder=False, text_to_image=True, aug_text=None,
                aug_image=None):
        """``CTCLIP.forward`` (ct_clip/ct_clip.py:614-901)."""
        if aug_text is not None or aug_image is not None:
            raise NotImplementedError('multiview augmentation is off in the reference configuration')
        if self.extra_latent_projection:
            raise NotImplementedError('extra_latent_projection (CLOOB) is off in the reference configuration')
        if return_latents:
            enc_text = self.text_transformer(text.input_ids, attention_mask=text.attention_mask)[0]
            tokens = self.visual_transformer(image, return_encoded_tokens=True)
            pooled, pooled_b = self._pool_tokens(tokens)
            t_raw = Fn.TextProjFn.apply(enc_text[:, 0, :].contiguous(), self.to_text_latent.weight)
            W = self.to_visual_latent.weight
            i_raw = self._project(W, self._visual_weight_bf16(W), pooled, pooled_b)
            return l2norm(t_raw), l2norm(i_raw), tokens
        self._t_gather = None
        enc_text, pooled, t_raw, i_raw = self.encode(text, image, gather=return_loss and not return_encodings)
        if return_encodings:
            return enc_text, pooled
        if not return_loss:
            from . import kernels as K
            return K.clip_scores(t_raw.contiguous(), i_raw.contiguous(), self.temperature.detach().reshape(1))
        tg, self._t_gather = self._t_gather, None
        return Fn.ClipLossFn.apply(t_raw, i_raw, self.temperature, None, tg)

    def backward_deferred_text(self):
        """Back-propagate the text tower whose graph ``encode`` detached (defer_text_backward).
        On the text stream, after the event the loss's backward recorded for its gradient: the
        autograd engine then sees producer and consumer on the same stream and adds no wait on the
        main stream (which would serialise BERT after the whole 3D-ViT backward)."""
        d, self._deferred_text = self._deferred_text, None
        if d is None or d[1].grad is None:
            return
        t_raw, leaf, ev = d
        g = leaf.grad
        ts = streams.text_stream(g.device)
        if ts is None or ev is None:
            torch.autograd.backward(t_raw, g)
            return
        ts.wait_event(ev)
        g.record_stream(ts)
        with torch.cuda.stream(ts):
            torch.autograd.backward(t_raw, g)

    def backward_deferred_image(self):
        """Back-propagate the image tower whose graph ``encode`` detached (after BERT's, see
        CTClipTrainer.forward_backward), on the current stream."""
        d, self._deferred_image = self._deferred_image, None
        if d is None or d[1].grad is None:
            return
        torch.autograd.backward(d[0], d[1].grad)

    def grad_buckets(self, text_first=True):
        """Gradient all-reduce buckets in the order the backward finalises them (dist_sync): BERT's
        layer groups from the top down (its backward is queued first, CTClipTrainer.forward_backward),
        the 3D-ViT's temporal stack, spatial stack, the rest of the image tower (patch embed, CPB),
        then the CTCLIP-level heads (projections, temperature), launched last."""
        vt = self.visual_transformer
        tb = getattr(self.text_transformer, 'grad_buckets', None)
        text = tb() if tb is not None else [('text_0', list(self.text_transformer.parameters()))]
        vit = [('vit_temporal', list(vt.enc_temporal_transformer.parameters())),
               ('vit_spatial', list(vt.enc_spatial_transformer.parameters())),
               ('vit_rest', list(vt.parameters()))]
        head = [('head', list(self.parameters()))]
        return text + vit + head if text_first else vit + text + head

    def _pool_tokens(self, tokens):
        """mean over t + flatten of already-quantised tokens (ct_clip.py:724,740)."""
        from . import kernels as K
        pooled = tokens.mean(dim=1).reshape(tokens.shape[0], -1)
        return pooled, K.cast_bf16(pooled.detach().contiguous())
