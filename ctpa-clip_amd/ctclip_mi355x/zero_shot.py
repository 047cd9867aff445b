"""Zero-shot pathology classification on the HIP path:
``ct_clip/ctclip_inference.py:261-338`` (``CTClipInference.train_step``).

The reference loops volume x pathology: for each of the 18 pathologies it tokenises the pair
("<p> is present.", "<p> is not present.") to 512 tokens, calls ``CTCLIP.forward(text, volume)``
in eval mode (``einsum('b d, b d -> b') * temp`` with the one volume broadcast over the two
prompts, ``ct_clip.py:805-807``), applies ``softmax(dim=0)`` (``ctclip_inference.py:92-104``) and
keeps entry 0 (``:312-315``) -- 18 image-tower encodes and 18 BERT passes per volume.

Here the work is factored without changing a number (eval mode is deterministic):
  * the 2P prompt latents are encoded ONCE (one BERT batch) and cached;
  * each volume batch goes through the image tower + projection ONCE;
  * one HIP kernel (``ctclip_zero_shot``) normalises, scores every (volume, prompt) pair and
    takes the pairwise softmax -> probs [N, P] (the reference's ``predictedall``).
"""
from __future__ import annotations

import torch

from . import functional as Fn
from . import kernels as K

# ct_clip/ctclip_inference.py:286-290
PATHOLOGIES = ('Medical material', 'Arterial wall calcification', 'Cardiomegaly', 'Pericardial effusion',
               'Coronary artery wall calcification', 'Hiatal hernia', 'Lymphadenopathy', 'Emphysema',
               'Atelectasis', 'Lung nodule', 'Lung opacity', 'Pulmonary Embolism', 'Pleural effusion',
               'Mosaic attenuation pattern', 'Peribronchial thickening', 'Consolidation', 'Bronchiectasis',
               'Interlobular septal thickening')


def prompts(pathologies=PATHOLOGIES):
    """The prompt pairs of ``ctclip_inference.py:306``, flattened: rows 2j / 2j+1."""
    out = []
    for p in pathologies:
        out += [f'{p} is present.', f'{p} is not present.']
    return out


class ZeroShotClassifier:
    """``predict(volumes) -> (probs [N, P], scores [N, P, 2])`` for a ``ctclip_mi355x.CTCLIP``.

    Prompts: either ``tokenizer`` (an HF tokenizer, called as the reference does with
    ``padding='max_length', truncation=True, max_length=512``) or pre-tokenised ``text`` (any
    object with ``.input_ids`` / ``.attention_mask`` of 2P rows) via ``set_prompts``."""

    def __init__(self, model, pathologies=PATHOLOGIES, tokenizer=None, max_length=512):
        self.model = model
        self.pathologies = tuple(pathologies)
        self.max_length = max_length
        self._t_raw = None
        if tokenizer is not None:
            dev = next(model.parameters()).device
            self.set_prompts(tokenizer(prompts(self.pathologies), return_tensors='pt', padding='max_length',
                                       truncation=True, max_length=max_length).to(dev))

    def set_prompts(self, text):
        ids = text.input_ids
        if ids.shape[0] != 2 * len(self.pathologies):
            raise ValueError(f'expected {2 * len(self.pathologies)} prompt rows (a present / not present pair '
                             f'per pathology), got {ids.shape[0]}')
        m = self.model
        with torch.no_grad(), _eval(m):
            enc = m.text_transformer(ids, attention_mask=text.attention_mask)[0]
            self._t_raw = Fn.TextProjFn.apply(enc[:, 0, :].contiguous(), m.to_text_latent.weight)
        return self

    def image_latents(self, volumes):
        """Raw projected image latents [N, Dl] (image tower + VQ + pool + to_visual_latent)."""
        m = self.model
        with torch.no_grad(), _eval(m):
            pooled, pooled_b = m.visual_transformer.encode_pooled(volumes)
            W = m.to_visual_latent.weight
            return m._project(W, m._visual_weight_bf16(W), pooled, pooled_b)

    def predict(self, volumes, batch_size=8):
        if self._t_raw is None:
            raise RuntimeError('ZeroShotClassifier: no prompts (pass tokenizer= or call set_prompts)')
        log_temp = self.model.temperature.detach().reshape(1)
        probs, scores = [], []
        for i in range(0, volumes.shape[0], batch_size):
            p, s = K.zero_shot(self._t_raw, self.image_latents(volumes[i:i + batch_size]), log_temp)
            probs.append(p)
            scores.append(s)
        return torch.cat(probs), torch.cat(scores)


class _eval:
    """Eval mode for the duration (the VQ codebook must not EMA-update during inference)."""

    def __init__(self, m):
        self.m = m

    def __enter__(self):
        self.was = self.m.training
        self.m.eval()

    def __exit__(self, *exc):
        self.m.train(self.was)
