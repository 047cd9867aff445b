"""Pin the CPU oracle (oracle/ctclip_oracle.py) against fixtures produced by the reference's
own ct_clip modules (tests/golden/make_golden.py).  CPU only."""
import numpy as np
import pytest
import torch

from oracle import ctclip_oracle as O
from oracle import weights as W


def _close(a, b, tol):
    a, b = a.double(), b.double()
    err = (a - b).abs().max().item()
    scale = max(1.0, b.abs().max().item())
    assert err <= tol * scale, f'max err {err} (scale {scale})'


def test_hu_division_bit_exact():
    """f32 x/1000.f == f64 divide-then-cast for every int16."""
    x = np.arange(-32768, 32768, dtype=np.int64)
    c = np.clip(x, -1000, 1000)
    ref = (c.astype(np.float64) / 1000).astype(np.float32)
    ours = O.normalize_hu(torch.from_numpy(x.astype(np.int16))).numpy()
    assert np.array_equal(ref.view(np.uint32), ours.view(np.uint32))


def test_recipe_is_deterministic():
    a = W.make_state_dict(O.TINY)
    b = W.make_state_dict(O.TINY)
    assert all(torch.equal(a[k], b[k]) for k in a)


def _run_tiny(golden, training=True, grads=False):
    cfg = O.TINY
    sd = W.make_state_dict(cfg)
    if grads:
        for k, v in sd.items():
            if k.startswith(O.trainable_prefixes()) and v.is_floating_point() and 'vq._codebook' not in k \
                    and not k.endswith('norm.beta') and not k.endswith('norm_out.beta') \
                    and not k.endswith('context_norm.beta'):
                v.requires_grad_(True)
    video = O.normalize_hu(golden['in.hu'])
    trace = {}
    out = O.ctclip_forward(sd, golden['in.ids'], golden['in.mask'], video, cfg, training, trace)
    return sd, out, trace


def test_tiny_forward_matches_reference(golden_tiny):
    g = golden_tiny
    assert torch.equal(g['in.hu'], W.make_hu(4, O.TINY.vit))
    sd, out, trace = _run_tiny(g)
    _close(trace['patch_emb'], g['out.patch_emb'], 1e-5)
    _close(trace['cpb'], g['out.cpb'], 1e-5)
    _close(trace['spatial_out'], g['out.spatial_out'].reshape(trace['spatial_out'].shape), 1e-4)
    _close(trace['temporal_out'],
           g['out.temporal_out'].reshape(4, 4, 4, 8, 64).permute(0, 3, 1, 2, 4), 1e-4)
    assert torch.equal(out['indices'], g['out.vq_indices'])
    _close(out['enc_text'], g['out.enc_text'], 1e-4)
    _close(out['loss'].reshape(1), g['out.loss'], 1e-5)
    _close(out['new_embed'], g['out.new_embed'], 1e-5)
    _close(out['new_cluster_size'], g['out.new_cluster_size'], 1e-6)


def test_tiny_grads_match_reference(golden_tiny):
    g = golden_tiny
    sd, out, _ = _run_tiny(g, grads=True)
    out['loss'].backward()
    n = 0
    for k in g:
        if not k.startswith('grad.'):
            continue
        name = k[5:]
        if g[k].numel() == 0:
            continue
        assert sd[name].grad is not None, name
        _close(sd[name].grad, g[k], 2e-4)
        n += 1
    assert n > 50


def test_tiny_eval_scores(golden_tiny):
    g = golden_tiny
    sd = W.make_state_dict(O.TINY)
    s = O.eval_scores(sd, g['in.ids'], g['in.mask'], O.normalize_hu(g['in.hu']), O.TINY)
    _close(s, g['out.eval_scores'], 1e-5)


@pytest.mark.slow
def test_base_b2_matches_reference(golden_base):
    g = golden_base
    cfg = O.BASE
    torch.set_num_threads(max(1, torch.get_num_threads()))
    sd = W.make_state_dict(cfg)
    ids, mask = W.make_text(2, 128, cfg.bert.vocab_size)
    video = O.normalize_hu(W.make_hu(2, cfg.vit))
    trace = {}
    with torch.no_grad():
        out = O.ctclip_forward(sd, ids, mask, video, cfg, True, trace)
    _close(trace['patch_emb'].reshape(-1, 512)[:256], g['out.patch_emb_head'], 1e-4)
    _close(trace['cpb'][:, :4, :], g['out.cpb_rows'], 1e-5)
    _close(trace['spatial_out'].reshape(-1, 512)[:256], g['out.spatial_out_head'], 1e-3)
    tout = trace['temporal_out'].permute(0, 2, 3, 1, 4).reshape(-1, 512)[:256]
    _close(tout, g['out.temporal_out_head'], 1e-3)
    mism = (out['indices'].to(torch.int32) != g['out.vq_indices']).float().mean().item()
    assert mism < 1e-3, mism
    _close(out['loss'].reshape(1), g['out.loss'], 1e-4)


def test_zero_shot_matches_reference():
    """Zero-shot scoring (ct_clip/ctclip_inference.py:305-315, eval branch ct_clip.py:805-807):
    the oracle's restatement (one image encode per volume) against the reference's own
    per-volume x per-pathology loop (golden_zeroshot_tiny, tests/golden/make_golden.py --zero-shot)."""
    from safetensors.torch import load_file
    import os
    g = load_file(os.path.join(os.path.dirname(__file__), 'golden', 'golden_zeroshot_tiny.safetensors'))
    cfg = O.TINY
    sd = W.make_state_dict(cfg)
    probs, scores = O.zero_shot(sd, g['in.ids'], g['in.mask'], O.normalize_hu(g['in.hu']), cfg)
    _close(scores, g['out.scores'], 1e-5)
    _close(probs, g['out.probs'], 1e-6)
    assert O.PATHOLOGIES[11] == 'Pulmonary Embolism' and len(O.PATHOLOGIES) == 18


def test_recon_matches_reference():
    """VQ-VAE reconstruction (ct_clip/ctvit.py:333-451, use_vgg_and_gan=False):
    the oracle's decode + MSE against the reference's own forward(video, return_recons=True) and
    backward (golden_recon_tiny, tests/golden/make_golden.py --recon)."""
    from safetensors.torch import load_file
    import os
    g = load_file(os.path.join(os.path.dirname(__file__), 'golden', 'golden_recon_tiny.safetensors'))
    cfg = O.TINY
    sd = W.make_state_dict(cfg)
    p = 'visual_transformer.'
    for k, v in sd.items():
        if ('grad.' + k) in g:
            v.requires_grad_(True)
    loss, recon, ind, _, _ = O.ctvit_recon(sd, p, O.normalize_hu(g['in.hu']), cfg.vit, training=True)
    assert torch.equal(ind.reshape(g['out.vq_indices'].shape), g['out.vq_indices'])
    _close(loss.detach().reshape(1), g['out.loss'], 1e-5)
    _close(recon.detach(), g['out.recon'], 1e-5)
    loss.backward()
    n = 0
    for k, v in sd.items():
        if ('grad.' + k) in g and v.grad is not None:
            _close(v.grad, g['grad.' + k], 2e-4)
            n += 1
    assert n >= 40, n


def test_vision_features_match_reference():
    """VisionFeatureExtractor (configs[4], ctpa_report/vqa_meditron.py:91-123): the oracle's
    vision_features against the reference's own to_patch_emb / enc_spatial_transformer (with the
    video_shape repair) + pooling + projector (golden_vfe, tests/golden/make_golden.py --vfe)."""
    from safetensors.torch import load_file
    import os
    g = load_file(os.path.join(os.path.dirname(__file__), 'golden', 'golden_vfe.safetensors'))
    vit = O.VFE_VIT
    sd = W.make_state_dict(O.ClipConfig(vit=vit, bert=O.TINY.bert, dim_latent=512))
    trace = {}
    with torch.no_grad():
        f = O.vision_features(sd, 'visual_transformer.', O.normalize_hu(W.make_hu(2, vit, seed=31)), vit,
                              W.make_projector(), trace=trace)
    _close(trace['patch_emb'], g['out.patch_emb'], 1e-5)
    _close(trace['spatial_out'], g['out.spatial_out'], 1e-5)
    _close(trace['pooled'], g['out.pooled'], 1e-5)
    _close(f, g['out.features'], 1e-5)
    assert f.shape == (2, 512)
