"""CTViT encoder path (ct_clip/ctvit.py:117-436) on HIP kernels.

Parameter / buffer layout matches the reference's ``CTViT.state_dict()`` (built with
``use_vgg_and_gan=False``), so ``CT-CLIP_v2.pt``-style checkpoints load unchanged.
"""
from __future__ import annotations

import os

import torch
from torch import nn

from . import dist_sync
from . import streams
from . import functional as Fn
from . import kernels as K
from .attention import ContinuousPositionBias, Transformer
from .layers import patch_offsets

_CPB_AUX = os.environ.get('CTCLIP_CPB_AUX', '1') != '0'
_PREPACK_AUX = os.environ.get('CTCLIP_PREPACK_AUX', '1') != '0'


def pair(v):
    return (v, v) if not isinstance(v, tuple) else v


class _Codebook(nn.Module):
    def __init__(self, dim, codebook_size):
        super().__init__()
        self.register_buffer('initted', torch.ones(1))
        self.register_buffer('cluster_size', torch.zeros(1, codebook_size))
        embed = nn.functional.normalize(nn.init.kaiming_uniform_(torch.empty(1, codebook_size, dim)), dim=-1)
        self.register_buffer('embed', embed)


class VectorQuantize(nn.Module):
    """Cosine-similarity VQ with EMA codebook (vector_quantize_pytorch==1.1.2 semantics as
    restated in oracle/ctclip_oracle.vq_forward; buffer names ``_codebook.{initted,cluster_size,embed}``)."""

    def __init__(self, dim, codebook_size, use_cosine_sim=True, decay=0.8, commitment_weight=1.):
        super().__init__()
        if not use_cosine_sim:
            raise NotImplementedError('only the cosine-similarity codebook is on the CT-CLIP path')
        self.dim = dim
        self.codebook_size = codebook_size
        self.decay = decay
        self._codebook = _Codebook(dim, codebook_size)
        self.state = Fn.VQState()

    @property
    def codebook(self):
        return self._codebook.embed[0]

    # The training step's codebook EMA runs on the auxiliary stream, possibly deferred past the
    # optimizer step (ct_clip.DEFER_EMA): every torch-API reader / writer of the codebook buffers is
    # ordered after it here, so a state_dict (checkpoint) holds the updated codebook and a load is not
    # overwritten by an EMA still in flight.  A pending (not yet queued) update is applied before a
    # save, and dropped by a load -- the loaded codebook replaces the state it would have updated.
    def _join_ema(self):
        dev = self._codebook.embed.device
        if dev.type == 'cuda':
            from . import streams
            streams.join_aux(dev)

    def state_dict(self, *args, **kwargs):
        self.state.flush_ema()
        self._join_ema()
        return super().state_dict(*args, **kwargs)

    def _load_from_state_dict(self, *args, **kwargs):
        self.state.pending_ema = None
        self._join_ema()
        return super()._load_from_state_dict(*args, **kwargs)


class _Slot(nn.Module):
    """Parameter-free placeholder keeping Sequential indices identical to the reference (Rearrange)."""


class CTViT(nn.Module):
    def __init__(self, *, dim, codebook_size, image_size, patch_size, temporal_patch_size, spatial_depth,
                 temporal_depth, discr_base_dim=16, dim_head=64, heads=8, channels=1, use_vgg_and_gan=False,
                 vgg=None, discr_attn_res_layers=(16,), use_hinge_loss=True, attn_dropout=0., ff_dropout=0.):
        super().__init__()
        if use_vgg_and_gan:
            raise NotImplementedError('VGG / GAN reconstruction losses are outside the contrastive hot path '
                                      '(ct_clip/ctvit.py:199-219); build with use_vgg_and_gan=False')
        if dim_head not in (32, 64):
            raise NotImplementedError('HIP attention kernels support dim_head 32 or 64')
        self.image_size = pair(image_size)
        self.patch_size = pair(patch_size)
        ph, pw = self.patch_size
        if ph != pw:
            raise NotImplementedError('square patches only')
        self.temporal_patch_size = temporal_patch_size
        self.dim = dim
        self.heads = heads
        self.dim_head = dim_head
        self.channels = channels
        self.spatial_rel_pos_bias = ContinuousPositionBias(dim=dim, heads=heads)
        pdf = channels * ph * pw
        pd = pdf * temporal_patch_size
        self.to_patch_emb_first_frame = nn.Sequential(_Slot(), nn.LayerNorm(pdf), nn.Linear(pdf, dim),
                                                      nn.LayerNorm(dim))
        self.to_patch_emb = nn.Sequential(_Slot(), nn.LayerNorm(pd), nn.Linear(pd, dim), nn.LayerNorm(dim))
        kw = dict(dim_head=dim_head, heads=heads, peg=True, peg_causal=True)
        self.enc_spatial_transformer = Transformer(dim, depth=spatial_depth, **kw)
        self.enc_temporal_transformer = Transformer(dim, depth=temporal_depth, **kw)
        self.enc_spatial_transformer.ready_tag = 'vit_spatial'     # gradient buckets (dist_sync)
        self.enc_temporal_transformer.ready_tag = 'vit_temporal'
        self.vq = VectorQuantize(dim=dim, codebook_size=codebook_size, use_cosine_sim=True)
        self.to_pixels_first_frame = nn.Sequential(nn.Linear(dim, pdf), _Slot())
        self.to_pixels = nn.Sequential(nn.Linear(dim, pd), _Slot())
        self.use_vgg_and_gan = False
        self._offs = {}

    @property
    def patch_height_width(self):
        return self.image_size[0] // self.patch_size[0], self.image_size[1] // self.patch_size[1]

    def _offsets(self, shape, device):
        key = (tuple(shape), str(device))
        if key not in self._offs:
            _, C, F, H, W = shape
            self._offs[key] = patch_offsets(C, self.temporal_patch_size, self.patch_size[0], F, H, W).to(device)
        return self._offs[key]

    # ------------------------------------------------------------------ encoder
    def encode_tokens(self, video, trace=None):
        """Patch-embed + spatial + temporal transformers.  video: (B, C, F, H, W) float in [-1, 1]
        or int16 HU (normalised in-kernel).  Returns (z f32 [M, D], z bf16, geometry); ``trace``
        (a dict, tests) receives the f32 token rows after patch-embed / spatial / temporal stacks."""
        # (the f32 image-tower mode, precise.py, runs inside the same Functions: functional.precise_f32)
        if video.ndim == 4:
            video = video.unsqueeze(2)
        assert video.ndim == 5
        B, C, F, H, W = video.shape
        assert (H, W) == tuple(self.image_size), (H, W)
        assert F % self.temporal_patch_size == 0
        is_hu = video.dtype == torch.int16
        if not is_hu and video.dtype != torch.float32:
            video = video.float()
        video = video.contiguous()
        hg, wg = self.patch_height_width
        # the CPB MLP (ctvit.py:317; ~0.14 ms of latency-bound f32 GEMMs forward, ~0.28 ms backward)
        # runs on the auxiliary stream beside the HBM-bound patch embedding; autograd runs its
        # backward there too (the stream of its forward), beside the patch-embed backward.  Its
        # parameter gradients are joined before the optimizer (trainer.optimizer_step: join_aux) and
        # before the image tower's bucket all-reduce (dist_sync).  CTCLIP_CPB_AUX=0: inline.
        dev = video.device
        aux = streams.aux_stream(dev) if _CPB_AUX else None
        cpb_ev = None
        if aux is not None:
            main = torch.cuda.current_stream(dev)
            aux.wait_stream(main)            # the previous optimizer step's update of the MLP
            with torch.cuda.stream(aux):
                bias_u = self.spatial_rel_pos_bias(hg, wg)
                # the layers' packed FeedForward weights too (16 small launches off the main stream)
                packs = Fn.prepack_ff(self._ff_weights(), self._out_weights(), self._qkv_weights()) \
                    if _PREPACK_AUX else []
                cpb_ev = aux.record_event()
            bias_u.record_stream(main)
            for t in packs:
                t.record_stream(main)
            node = bias_u.grad_fn
            if node is not None:
                def cpb_ready(du, node=node, aux=aux):
                    # called by the last spatial layer's backward right after its attention backward
                    # (functional._bias_grad_ready): the CPB MLP's backward starts there, on aux
                    aux.wait_stream(torch.cuda.current_stream(du.device))
                    with torch.cuda.stream(aux):
                        Fn.CPBFn.backward(node, du)
                    du.record_stream(aux)
                    node._ctclip_done = True
                bias_u.__dict__['_ctclip_bias_acc'] = {'n': 0, 'du': None, 'ready': cpb_ready}
        pe = self.to_patch_emb
        xf, xb = Fn.PatchEmbedFn.apply(video, pe[1].weight, pe[1].bias, pe[2].weight, pe[2].bias, pe[3].weight,
                                       pe[3].bias, self.temporal_patch_size, self.patch_size[0], is_hu,
                                       self._offsets(video.shape, video.device))
        dist_sync.mark_ready(xf, 'vit_rest')   # with the CPB node below: the rest of the image tower
        streams.mark_image_head(video.device)   # deferred text-stream work may start (streams.py)
        if self.training:
            from . import ct_clip
            if ct_clip.DEFER_EMA == '3':
                self.vq.state.flush_ema()      # the previous step's codebook EMA (ct_clip.DEFER_EMA '3')
        # CTCLIP.encode may start BERT's forward only once the HBM-bound patch LayerNorm is done
        self._patch_done = torch.cuda.current_stream(dev).record_event() if dev.type == 'cuda' else None
        if trace is not None:
            trace['patch_emb'] = xf
        T = F // self.temporal_patch_size
        g_sp = Fn.Geo(B, T, hg, wg, self.heads, self.dim_head, 0)
        g_tm = Fn.Geo(B, T, hg, wg, self.heads, self.dim_head, 1)
        if cpb_ev is not None:
            torch.cuda.current_stream(dev).wait_event(cpb_ev)
        else:
            bias_u = self.spatial_rel_pos_bias(hg, wg)                   # ctvit.py:317
        dist_sync.mark_ready(bias_u, 'vit_rest')
        xf, xb = self.enc_spatial_transformer.run(xf, xb, g_sp, bias_u)   # ctvit.py:319
        zf, zb = self.enc_temporal_transformer.run(xf, xb, g_tm)         # ctvit.py:327
        if trace is not None:
            trace['spatial_out'], trace['temporal_out'] = xf, zf
        return zf, zb, g_sp

    def _out_weights(self):
        return [attn.to_out.weight for tr in (self.enc_spatial_transformer, self.enc_temporal_transformer)
                for (_, attn, _, _) in tr.layers]

    def _qkv_weights(self):
        """(Wq, LayerNorm gamma, Wkv, q_scale, k_scale) of every layer whose Q | K | V projection
        folds its LayerNorm (functional.ViTLayerFn; the fold's own gate decides per layer, an
        unused prepack is dropped at the next one)"""
        if not Fn._LN1_FOLD or self.dim_head != 32 or self.heads * self.dim_head != 256:
            return []
        return [(attn.to_q.weight, attn.norm.gamma, attn.to_kv.weight, attn.q_scale, attn.k_scale)
                for tr in (self.enc_spatial_transformer, self.enc_temporal_transformer)
                for (_, attn, _, _) in tr.layers]

    def _ff_weights(self):
        return [(ff[1].weight, ff[4].weight) for tr in (self.enc_spatial_transformer, self.enc_temporal_transformer)
                for (_, _, _, ff) in tr.layers]

    def encode_pooled(self, video):
        """Encoder + VQ + mean over t (the CTCLIP image path, ct_clip.py:715,724,740):
        returns (pooled f32 [B, h*w*d], pooled bf16)."""
        zf, zb, geo = self.encode_tokens(video)
        cb = self._codebook_tensors()
        pooled, pooled_b, _ = Fn.VQPoolFn.apply(zf, zb, cb[0], cb[1], geo, self.training, self.vq.decay,
                                                self.vq.state, False)
        return pooled, pooled_b

    def _codebook_tensors(self):
        self.vq.state.flush_ema()        # a deferred EMA update (CTCLIP.encode) precedes any read
        c = self.vq._codebook
        return c.embed, c.cluster_size

    def _decode_rows(self, zf, geo):
        """CTViT.decode (ct_clip/ctvit.py:333-366) on canonical token rows: the encoder's temporal
        then spatial transformers again (same raw-reshape PEG view, CPB bias) -> (f32, bf16)."""
        xf, xb = zf, K.cast_bf16(zf.detach())
        g_tm = Fn.Geo(geo.B, geo.T, geo.Hg, geo.Wg, self.heads, self.dim_head, 1)
        xf, xb = self.enc_temporal_transformer.run(xf, xb, g_tm)
        bias_u = self.spatial_rel_pos_bias(geo.Hg, geo.Wg)
        dist_sync.mark_ready(bias_u, 'vit_rest')
        return self.enc_spatial_transformer.run(xf, xb, geo, bias_u)

    def decode(self, tokens):
        """``CTViT.decode`` (ct_clip/ctvit.py:333-375): tokens (b, t, h, w, d) or (b, t*h*w, d)
        -> reconstructed video (b, c, t*pt, h*p1, w*p2) f32."""
        hg, wg = self.patch_height_width
        b = tokens.shape[0]
        z = tokens.reshape(-1, self.dim).float().contiguous()
        T = z.shape[0] // (b * hg * wg)
        geo = Fn.Geo(b, T, hg, wg, self.heads, self.dim_head, 0)
        xf, xb = self._decode_rows(z, geo)
        W, bias = self.to_pixels[0].weight, self.to_pixels[0].bias
        Wb = Fn.bf(W)
        pix = K.linear(xb, Wb, bias=bias, out_dtype=torch.float32)
        c, pt, p = self.channels, self.temporal_patch_size, self.patch_size[0]
        # Rearrange 'b t h w (c pt p1 p2) -> b c (t pt) (h p1) (w p2)' (ctvit.py:196)
        return (pix.view(b, T, hg, wg, c, pt, p, p).permute(0, 4, 1, 5, 2, 6, 3, 7)
                .reshape(b, c, T * pt, hg * p, wg * p))

    def forward(self, video, mask=None, return_recons=False, return_recons_only=False, return_discr_loss=False,
                apply_grad_penalty=True, return_only_codebook_ids=False, return_encoded_tokens=False):
        """``CTViT.forward`` (ct_clip/ctvit.py:377-451): the encoder path (return_encoded_tokens /
        return_only_codebook_ids) and, with ``use_vgg_and_gan=False``, the VQ-VAE reconstruction
        path (MSE loss; return_recons / return_recons_only)."""
        if mask is not None:
            raise NotImplementedError('frame masks are not used on the CT-CLIP path')
        if return_discr_loss or self.use_vgg_and_gan:
            raise NotImplementedError('the GAN / perceptual losses (VGG16 weights) are out of scope')
        if video.ndim == 4:
            video = video.unsqueeze(2)
        zf, zb, geo = self.encode_tokens(video)
        emb, cs = self._codebook_tensors()
        want_tokens = not return_only_codebook_ids
        _, _, toks = Fn.VQPoolFn.apply(zf, zb, emb, cs, geo, self.training, self.vq.decay, self.vq.state,
                                       want_tokens)
        if return_only_codebook_ids:
            return self.vq.state.last_indices.view(geo.B, -1).long()
        if return_encoded_tokens:
            return toks.view(geo.B, geo.T, geo.Hg, geo.Wg, self.dim)
        # reconstruction (ctvit.py:436-451): decode the quantised tokens, MSE against the input
        xf, xb = self._decode_rows(toks, geo)
        is_hu = video.dtype == torch.int16
        vid = video if is_hu else video.float().contiguous()
        want_recon = return_recons or return_recons_only
        loss, recon = Fn.ReconFn.apply(xf, xb, self.to_pixels[0].weight, self.to_pixels[0].bias, vid, is_hu,
                                       self.temporal_patch_size, self.patch_size[0],
                                       self._offsets(vid.shape, vid.device), want_recon)
        if return_recons_only:
            return recon
        if return_recons:
            return loss, recon
        return loss
