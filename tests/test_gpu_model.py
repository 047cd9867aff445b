"""End-to-end parity of the HIP contrastive step against the CPU oracle (GPU).

Config: the base CT-CLIP widths (ViT d=512, 8x32 heads, FF 1365, codebook 8192; BERT 768/12)
on a reduced volume (160x160x40 -> 4x8x8 tokens), 2+2 ViT layers and 2 BERT layers, so the
fp32 oracle finishes in seconds.  The vector quantiser's argmax is compared separately (index
agreement rate, near-ties allowed); everything downstream is compared with the oracle forced
onto the HIP path's indices (every index difference must be a near-tie explained by the token's
measured pre-VQ error).  Tolerances are bf16-path tolerances: latents and
loss within 1e-3, intermediate activations / gradients as stated per check."""
import types

import pytest
import torch

from oracle import ctclip_oracle as O
from oracle import weights as W

pytestmark = pytest.mark.gpu


def cfg_small():
    vit = O.ViTConfig(dim=512, codebook_size=8192, image_size=160, patch_size=20, temporal_patch_size=10,
                      spatial_depth=2, temporal_depth=2, dim_head=32, heads=8, frames=40)
    bert = O.BertConfig(vocab_size=1000, hidden=768, layers=2, heads=12, intermediate=3072, max_position=64)
    return O.ClipConfig(vit=vit, bert=bert, dim_latent=512)


def build(cfg, dropout=0.0):
    from ctclip_mi355x.models import build_ctclip, set_finetune_trainable
    from ctclip_mi355x.bert import BertConfig
    v, b = cfg.vit, cfg.bert
    vit = dict(dim=v.dim, codebook_size=v.codebook_size, image_size=v.image_size, patch_size=v.patch_size,
               temporal_patch_size=v.temporal_patch_size, spatial_depth=v.spatial_depth,
               temporal_depth=v.temporal_depth, dim_head=v.dim_head, heads=v.heads)
    bert = BertConfig(vocab_size=b.vocab_size, hidden_size=b.hidden, num_hidden_layers=b.layers,
                      num_attention_heads=b.heads, intermediate_size=b.intermediate,
                      max_position_embeddings=b.max_position,
                      hidden_dropout_prob=dropout, attention_probs_dropout_prob=dropout)   # parity runs: 0
    m = build_ctclip(vit, bert, cfg.dim_latent)
    m.load_state_dict(W.make_state_dict(cfg), strict=True)
    return set_finetune_trainable(m).cuda()


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.fixture(scope='module')
def setup():
    torch.manual_seed(0)
    cfg = cfg_small()
    model = build(cfg)
    B = 2
    hu = W.make_hu(B, cfg.vit)
    ids, mask = W.make_text(B, 32, cfg.bert.vocab_size, ragged=True)
    text = types.SimpleNamespace(input_ids=ids.cuda(), attention_mask=mask.cuda())
    return cfg, model, hu, ids, mask, text


def test_encoder_stages_match_oracle(setup):
    cfg, model, hu, ids, mask, text = setup
    sd = W.make_state_dict(cfg)
    video = O.normalize_hu(hu)
    vt = model.visual_transformer
    with torch.no_grad():
        trace = {}
        O.ctvit_encode(sd, 'visual_transformer.', O.patch_embed(sd, 'visual_transformer.', video, cfg.vit),
                       cfg.vit, trace)
        pe = O.patch_embed(sd, 'visual_transformer.', video, cfg.vit)
        zf, zb, geo = vt.encode_tokens(hu.cuda())
        # f32 video in [-1, 1] takes the same path bit-for-bit in the patch kernel
        zf2, _, _ = vt.encode_tokens(video.cuda())
    assert torch.equal(zf, zf2)
    r = rel(zf, trace['temporal_out'].reshape(-1, 512))
    print('pre-VQ tokens rel err', r)
    assert r < 2e-2
    u = vt.spatial_rel_pos_bias.dense(8, 8)
    assert rel(u, trace['cpb']) < 1e-5


def test_forward_latents_and_loss(setup):
    cfg, model, hu, ids, mask, text = setup
    sd = W.make_state_dict(cfg)
    video = O.normalize_hu(hu)
    model.eval()
    with torch.no_grad():
        enc_text, pooled, t_raw, i_raw = model.encode(text, hu.cuda())
        idx = model.visual_transformer.vq.state.last_indices.cpu()
        scores = model(text, hu.cuda(), return_loss=False)
        zf, _, _ = model.visual_transformer.encode_tokens(hu.cuda())
    trace = {}
    with torch.no_grad():
        free = O.ctclip_forward(sd, ids, mask, video, cfg, training=False, trace=trace)
        forced = O.ctclip_forward(sd, ids, mask, video, cfg, training=False, force_ind=idx)
    # VQ contract, margin-based: every index the bf16 path picks differently from the
    # oracle must be a near-tie its own pre-VQ error explains -- the oracle's score gap between its
    # winner and the HIP choice at most 2 * |l2norm(z_hip) - l2norm(z_oracle)| (both unit-code
    # scores move by at most that much); the count above the literal 1e-6 margin is reported (the
    # f32 image tower meets it literally: test_gpu_f32path.py, test_gpu_base.py)
    zo = trace['temporal_out'].reshape(-1, cfg.vit.dim)
    oi, hi = free['indices'].reshape(-1).long(), idx.long()
    diff = (oi != hi).nonzero().flatten()
    E = sd['visual_transformer.vq._codebook.embed'][0]
    xo = torch.nn.functional.normalize(zo, dim=-1)
    xh = torch.nn.functional.normalize(zf.cpu(), dim=-1)
    so = xo[diff] @ E.t()
    gap = so.gather(1, oi[diff][:, None]).squeeze(1) - so.gather(1, hi[diff][:, None]).squeeze(1)
    bound = 2 * (xh[diff] - xo[diff]).norm(dim=1)
    print(f'VQ: {diff.numel()} of {oi.numel()} indices differ, {(gap >= 1e-6).sum().item()} with oracle gap '
          f'>= 1e-6, max gap {gap.max().item() if diff.numel() else 0:.2e}; all within their token-error bound: '
          f'{bool((gap <= bound + 1e-6).all())}')
    assert (gap > bound + 1e-6).sum().item() == 0
    tl = torch.nn.functional.normalize(t_raw, dim=-1)
    il = torch.nn.functional.normalize(i_raw, dim=-1)
    assert (tl.cpu() - forced['text_latents']).abs().max().item() < 1e-3
    assert (il.cpu() - forced['image_latents']).abs().max().item() < 1e-3
    ref_scores = (forced['text_latents'] * forced['image_latents']).sum(-1) * torch.e
    assert (scores.cpu() - ref_scores).abs().max().item() < 1e-3
    model.train()


def test_backward_grads(setup):
    cfg, model, hu, ids, mask, text = setup
    sd = W.make_state_dict(cfg)
    video = O.normalize_hu(hu)
    model.train()
    emb0 = model.visual_transformer.vq._codebook.embed.clone()
    model.zero_grad(set_to_none=True)
    loss = model(text, hu.cuda(), return_loss=True)
    idx = model.visual_transformer.vq.state.last_indices.cpu()
    loss.backward()
    for k, v in sd.items():
        if k.startswith(('visual_transformer.', 'text_transformer.')) and v.is_floating_point() and \
                'vq._codebook' not in k and not k.endswith('beta') and v.numel():
            v.requires_grad_(True)
    out = O.ctclip_forward(sd, ids, mask, video, cfg, training=True, force_ind=idx)
    out['loss'].backward()
    assert abs(loss.item() - out['loss'].item()) < 1e-3
    # EMA codebook update on the same indices; the per-code means average the bf16-path tokens,
    # which are ~1e-2 off the oracle's, scaled by (1 - decay) = 0.2 (exact semantics on identical
    # inputs: tests/test_gpu_ops.py::test_vq_select_and_pool)
    assert rel(model.visual_transformer.vq._codebook.embed, out['new_embed']) < 5e-3
    named = dict(model.named_parameters())
    checks = {
        'visual_transformer.to_patch_emb.2.weight': 5e-2,
        'visual_transformer.to_patch_emb.1.weight': 5e-2,
        'visual_transformer.to_patch_emb.3.weight': 5e-2,
        'visual_transformer.spatial_rel_pos_bias.net.0.0.weight': 5e-2,
        'visual_transformer.spatial_rel_pos_bias.net.2.weight': 5e-2,
        'visual_transformer.enc_spatial_transformer.layers.0.0.dsconv.weight': 5e-2,
        'visual_transformer.enc_spatial_transformer.layers.0.1.to_q.weight': 5e-2,
        'visual_transformer.enc_spatial_transformer.layers.0.1.to_kv.weight': 5e-2,
        'visual_transformer.enc_spatial_transformer.layers.0.1.q_scale': 5e-2,
        'visual_transformer.enc_spatial_transformer.layers.1.3.1.weight': 5e-2,
        'visual_transformer.enc_spatial_transformer.layers.1.3.4.weight': 5e-2,
        'visual_transformer.enc_temporal_transformer.layers.0.0.dsconv.weight': 5e-2,
        'visual_transformer.enc_temporal_transformer.layers.1.1.to_out.weight': 5e-2,
        'visual_transformer.enc_temporal_transformer.norm_out.gamma': 5e-2,
        'text_transformer.embeddings.word_embeddings.weight': 5e-2,
        'text_transformer.encoder.layer.0.attention.self.query.weight': 5e-2,
        'text_transformer.encoder.layer.1.output.dense.weight': 5e-2,
        'text_transformer.encoder.layer.1.output.LayerNorm.bias': 5e-2,
    }
    bad = []
    for name, tol in checks.items():
        r = rel(named[name].grad, sd[name].grad)
        print(f'{name}: grad rel err {r:.2e}')
        if not r < tol:
            bad.append((name, r))
    assert not bad, bad
    model.visual_transformer.vq._codebook.embed.copy_(emb0)


def test_trainer_step_runs(setup):
    cfg, model, hu, ids, mask, text = setup
    from ctclip_mi355x.trainer import CTClipTrainer
    tr = CTClipTrainer(model, lr=1e-4)
    p = model.visual_transformer.enc_spatial_transformer.layers[0][1].to_q.weight
    before = p.detach().clone()
    l1 = tr.train_step(text, hu.cuda())
    l2 = tr.train_step(text, hu.cuda())
    torch.cuda.synchronize()
    assert torch.isfinite(l1) and torch.isfinite(l2)
    assert not torch.equal(before, p.detach())
    assert p.data_ptr() >= tr.flat.data.data_ptr()
    assert tr.norm[0].item() > 0
    # the Adam kernel's bf16 shadows (trainer.FlatParams) equal the RNE bf16 of every updated
    # weight, BERT's q / k / v come out of the shadow arena as one slice, and an in-place torch
    # update of a weight retires its shadow (the GEMMs then cast afresh)
    from ctclip_mi355x import functional as Fn
    for q in tr.flat.params:
        sh = Fn.shadow_bf16(q)
        assert sh is not None and torch.equal(sh, q.detach().bfloat16())
    a = model.text_transformer.encoder.layer[0].attention.self
    qkv = Fn.bf_cat([a.query.weight, a.key.weight, a.value.weight])
    assert qkv.data_ptr() == Fn.shadow_bf16(a.query.weight).data_ptr()
    assert torch.equal(qkv, torch.cat([a.query.weight, a.key.weight, a.value.weight]).detach().bfloat16())
    assert Fn.cat_f32([a.query.bias, a.key.bias, a.value.bias]).data_ptr() == a.query.bias.data_ptr()
    with torch.no_grad():
        p.add_(0.0)
    assert Fn.shadow_bf16(p) is None
    assert torch.equal(Fn.bf(p), p.detach().bfloat16())
    tr.train_step(text, hu.cuda())   # the next Adam step re-syncs it
    torch.cuda.synchronize()
    assert Fn.shadow_bf16(p) is not None


def test_grad_buckets_final_when_launched(setup):
    """Backward-overlapped gradient sync (dist_sync.BucketedGradSync): with the
    hooks forced on at world 1, each bucket's gradient slice at the moment its hook launches the
    all-reduce must already equal its final value (bit-exact), the hooks must fire in bucket
    order during the backward: BERT's layer groups from the top down (here one layer per bucket),
    queued first, then the 3D-ViT stacks and the rest of the image tower."""
    cfg, model, hu, ids, mask, text = setup
    from ctclip_mi355x.trainer import CTClipTrainer
    model.text_transformer.bucket_layers = 1
    tr = CTClipTrainer(model, lr=1e-4)
    gs = tr.grad_sync
    order = ['text_1', 'text_0', 'vit_temporal', 'vit_spatial', 'vit_rest']
    assert [t for t, _, _ in gs.buckets] == order
    snaps = {}
    fold = gs.before_launch

    def snap(tag):
        fold(tag)
        _, off, n = next(b for b in gs.buckets if b[0] == tag)
        snaps[tag] = tr.flat.grad[off:off + n].clone()
    gs.before_launch = snap
    gs.force = True
    tr.flat.grad.zero_()
    tr.forward_backward(text, hu.cuda())
    assert gs.launched == order, gs.launched
    gs.finish()
    torch.cuda.synchronize()
    for tag, off, n in gs.buckets:
        assert torch.equal(snaps[tag], tr.flat.grad[off:off + n]), tag
        assert snaps[tag].abs().sum().item() > 0, tag
    model.text_transformer.bucket_layers = 3


def test_zero_shot_matches_oracle(setup):
    """Zero-shot pathology scoring (ct_clip/ctclip_inference.py:305-315): the HIP path (prompt
    latents once, one image encode per volume, ctclip_zero_shot kernel) vs the oracle's loop,
    with the oracle forced onto the HIP path's VQ indices; probabilities / scores within 2e-3
    absolute (both towers compute in bf16 with f32 accumulation against the f32 oracle, on the
    weights left by the optimizer steps of the earlier tests: 0.3-1.5e-3 measured).
    Also the reference's direct call shape: 2 prompts x 1 volume broadcast -> (2,) scores."""
    cfg, model, hu, ids, mask, text = setup
    from ctclip_mi355x.zero_shot import ZeroShotClassifier, PATHOLOGIES
    P = 3
    pids, pmask = W.make_text(2 * P, 32, cfg.bert.vocab_size, seed=99, ragged=True)
    zs = ZeroShotClassifier(model, pathologies=PATHOLOGIES[:P])
    zs.set_prompts(types.SimpleNamespace(input_ids=pids.cuda(), attention_mask=pmask.cuda()))
    model.train()          # predict() must switch to eval (no EMA update) and restore the mode
    cb0 = model.visual_transformer.vq._codebook.embed.detach().clone()
    probs, scores = zs.predict(hu.cuda())
    idx = model.visual_transformer.vq.state.last_indices.cpu()
    assert model.training
    assert torch.equal(cb0, model.visual_transformer.vq._codebook.embed)
    torch.cuda.synchronize()
    # the model's CURRENT weights (earlier tests in this module take optimizer steps)
    sd = {k: v.detach().float().cpu() for k, v in model.state_dict().items()}
    with torch.no_grad():
        rp, rs = O.zero_shot(sd, pids, pmask, O.normalize_hu(hu), cfg, force_ind=idx.reshape(hu.shape[0], -1))
    assert probs.shape == (hu.shape[0], P) and scores.shape == (hu.shape[0], P, 2)
    assert (scores.cpu() - rs).abs().max().item() < 2e-3
    assert (probs.cpu() - rp).abs().max().item() < 2e-3
    # the reference's own per-pathology call: CTCLIP.forward(2 prompts, 1 volume) in eval mode
    model.eval()
    with torch.no_grad():
        pair = types.SimpleNamespace(input_ids=pids[:2].cuda(), attention_mask=pmask[:2].cuda())
        s2 = model(pair, hu[:1].cuda(), return_loss=False)
    model.train()
    assert s2.shape == (2,)
    assert (s2.cpu() - scores[0, 0].cpu()).abs().max().item() < 1e-4


def test_recon_matches_oracle(setup):
    """VQ-VAE reconstruction path (ct_clip/ctvit.py:333-451 with
    use_vgg_and_gan=False): CTViT.forward(video, return_recons=True) -> (MSE loss, recon) and its
    backward against the oracle's ctvit_recon, the oracle forced onto the HIP path's VQ indices and
    given the pre-step weights.  Loss within 1e-3 relative, recon 3e-2 (the pre-VQ tokens are within
    2e-2 after the 8 encoder layers; the decoder adds 8 more bf16 layers), grads within 5 %."""
    cfg, model, hu, ids, mask, text = setup
    vit = model.visual_transformer
    sd = {k: v.detach().float().cpu().clone() for k, v in model.state_dict().items()}
    for prm in vit.parameters():
        prm.grad = None
    px = list(vit.to_pixels.parameters())      # frozen on the contrastive path (set_finetune_trainable)
    for prm in px:
        prm.requires_grad_(True)
    vit.train()
    loss, recon = vit(hu.cuda(), return_recons=True)
    idx = vit.vq.state.last_indices.cpu()
    loss.backward()
    torch.cuda.synchronize()
    # the reference's return_recons_only / decode() agree with the fused path
    assert recon.shape == (hu.shape[0], 1, cfg.vit.frames, cfg.vit.image_size, cfg.vit.image_size)
    p = 'visual_transformer.'
    names = ['to_pixels.0.weight', 'to_pixels.0.bias', 'enc_spatial_transformer.layers.1.3.1.weight',
             'enc_temporal_transformer.layers.0.1.to_q.weight', 'to_patch_emb.2.weight']
    for n in names:
        sd[p + n].requires_grad_(True)
    rl, rr, _, _, _ = O.ctvit_recon(sd, p, O.normalize_hu(hu), cfg.vit, training=True,
                                    force_ind=idx.reshape(hu.shape[0], -1))
    rl.backward()
    assert abs(loss.item() - rl.item()) <= 1e-3 * abs(rl.item()), (loss.item(), rl.item())
    assert rel(recon, rr) < 3e-2, rel(recon, rr)     # 8 more bf16 transformer layers than the latents
    named = dict(vit.named_parameters())
    for n in names:
        r = rel(named[n].grad, sd[p + n].grad)
        print(f'{n}: grad rel err {r:.2e}')
        assert r < 5e-2, (n, r)
    for prm in vit.parameters():
        prm.grad = None
    for prm in px:
        prm.requires_grad_(False)
    # eval: the public decode() of the encoded tokens equals the fused return_recons_only path
    vit.eval()
    with torch.no_grad():
        r1 = vit(hu.cuda(), return_recons_only=True)
        r2 = vit.decode(vit(hu.cuda(), return_encoded_tokens=True))
    vit.train()
    assert torch.equal(r1, r2)


def test_deferred_text_adam_matches(setup):
    """trainer.defer_text_adam (the text bucket's Adam queued by the next step's BERT forward;
    streams.defer_text): three steps then flush give bit-identical losses and parameters to the
    immediate placement at the reduced parity config (8 x 8 spatial grid: the frame-inner dQ
    kernel's fixed-order bias binning; no float atomics on the step's path).  The ordering itself
    is checked by test_defer_text_ordering."""
    cfg, _, hu, ids, mask, text = setup
    from ctclip_mi355x.trainer import CTClipTrainer
    lr = 1e-4
    outs = []
    for defer in (False, True):
        torch.manual_seed(0)
        model = build(cfg)
        tr = CTClipTrainer(model, lr=lr, defer_text_adam=defer)
        losses = [tr.train_step(text, hu.cuda()) for _ in range(3)]
        tr.flush()
        torch.cuda.synchronize()
        outs.append((torch.stack(losses), tr.flat.data.clone()))
    (l0, p0), (l1, p1) = outs
    assert torch.equal(l0, l1)
    assert torch.equal(p0, p1), (p0 - p1).abs().max().item()


def test_state_dict_after_deferred_adam_is_current(setup):
    """CTCLIP.state_dict right after a step whose text Adam was deferred: copies of the
    returned tensors queued on the caller's stream -- what torch.save does -- hold the updated
    weights, not pre-update or torn ones (state_dict joins the text and auxiliary streams)."""
    cfg, _, hu, ids, mask, text = setup
    from ctclip_mi355x.trainer import CTClipTrainer
    torch.manual_seed(0)
    model = build(cfg)
    tr = CTClipTrainer(model, lr=1e-3, defer_text_adam=True)
    before = {k: v.detach().clone() for k, v in model.state_dict().items() if k.startswith('text_transformer.')}
    tr.train_step(text, hu.cuda())
    sd = model.state_dict()                       # no synchronize in between
    snap = {k: sd[k].detach().clone() for k in before}      # queued on the current stream
    torch.cuda.synchronize()
    final = model.state_dict()
    moved = 0
    for k in before:
        assert torch.equal(snap[k], final[k]), k
        moved += int(not torch.equal(before[k], final[k]))
    assert moved > 0


def test_load_after_train_step_keeps_checkpoint_codebook(setup, tmp_path):
    """the codebook EMA of a train_step runs on the auxiliary stream after the optimizer
    step (ct_clip.DEFER_EMA '2').  A checkpoint loaded right after the step -- no synchronize -- must
    end with exactly the checkpoint's codebook (the load joins the EMA first and drops a pending
    one), and a state_dict taken right after a step holds the updated codebook."""
    cfg, _, hu, ids, mask, text = setup
    from ctclip_mi355x.trainer import CTClipTrainer
    torch.manual_seed(0)
    model = build(cfg)
    ck = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    path = tmp_path / 'ck.pt'
    torch.save(ck, str(path))
    tr = CTClipTrainer(model, lr=1e-4)
    cbk = model.visual_transformer.vq._codebook
    for _ in range(2):
        tr.train_step(text, hu.cuda())
        model.load(str(path))                     # no synchronize in between
        torch.cuda.synchronize()
        assert torch.equal(cbk.embed.cpu(), ck['visual_transformer.vq._codebook.embed'])
        assert torch.equal(cbk.cluster_size.cpu(), ck['visual_transformer.vq._codebook.cluster_size'])
    tr.train_step(text, hu.cuda())
    snap = model.state_dict()['visual_transformer.vq._codebook.embed'].clone()   # queued, no sync
    torch.cuda.synchronize()
    assert torch.equal(snap, cbk.embed)
    assert not torch.equal(snap.cpu(), ck['visual_transformer.vq._codebook.embed'])


def test_train_step_bit_reproducible():
    """Two runs of three training steps from the same seed give bit-identical losses, parameters,
    Adam moments, VQ codebook and cluster sizes, BERT dropout on, ragged reports (pad ids): no
    float atomics on the step's path (CPB bias gradient through the per-workgroup workspace,
    embedding and patch-LN gradients in fixed order, VQ statistics in fixed point).  A third run
    with the text Adam deferred (trainer.defer_text_adam) is bit-identical too, and so is a fourth
    with the CPB MLP inline on the main stream instead of the auxiliary one (ctvit._CPB_AUX), and a
    fifth and sixth with the codebook EMA queued right after the VQ / after the projection instead
    of after the optimizer step (ct_clip.DEFER_EMA).  The
    spatial stage runs the base shape (24 x 24 grid, L = 576: the LDS-DMA dQ kernel); smaller grids
    take the frame-inner kernel, checked by test_deferred_text_adam_matches."""
    from ctclip_mi355x.trainer import CTClipTrainer
    from ctclip_mi355x import ctvit
    vit = O.ViTConfig(dim=512, codebook_size=8192, image_size=480, patch_size=20, temporal_patch_size=10,
                      spatial_depth=1, temporal_depth=1, dim_head=32, heads=8, frames=20)
    bert = O.BertConfig(vocab_size=1000, hidden=768, layers=2, heads=12, intermediate=3072, max_position=64)
    cfg = O.ClipConfig(vit=vit, bert=bert, dim_latent=512)
    torch.manual_seed(1)
    hu = W.make_hu(2, cfg.vit).cuda()
    ids, mask = W.make_text(2, 32, bert.vocab_size, ragged=True)
    assert (ids == 0).any()
    text = types.SimpleNamespace(input_ids=ids.cuda(), attention_mask=mask.cuda())
    from ctclip_mi355x import ct_clip
    runs = []
    cpb_aux, dema = ctvit._CPB_AUX, ct_clip.DEFER_EMA
    for defer, aux, de in ((False, cpb_aux, dema), (False, cpb_aux, dema), (True, cpb_aux, dema),
                           (False, not cpb_aux, dema), (False, cpb_aux, '0'), (False, cpb_aux, '1')):
        torch.manual_seed(0)
        ctvit._CPB_AUX = aux
        ct_clip.DEFER_EMA = de
        model = build(cfg, dropout=0.1)
        tr = CTClipTrainer(model, lr=1e-4, defer_text_adam=defer)
        try:
            losses = torch.stack([tr.train_step(text, hu) for _ in range(3)])
            tr.flush()
        finally:
            ctvit._CPB_AUX = cpb_aux
            ct_clip.DEFER_EMA = dema
        torch.cuda.synchronize()
        cbk = model.visual_transformer.vq._codebook
        runs.append([losses, tr.flat.data.clone(), tr.m.clone(), tr.v.clone(), cbk.embed.clone(),
                     cbk.cluster_size.clone()])
        del model, tr
    names = ['losses', 'parameters', 'adam m', 'adam v', 'codebook', 'cluster size']
    for i, r in enumerate(runs[1:], 1):
        for n, a, b in zip(names, runs[0], r):
            assert torch.equal(a, b), f'run {i}: {n} differ: max {(a.double() - b.double()).abs().max().item():.3e}'
    assert torch.isfinite(runs[0][0]).all()


def test_defer_text_ordering():
    """streams.defer_text / mark_image_head / flush_text order deferred work after the main-stream
    work queued before the deferral (the clip coefficient), after the marked point of the next
    forward, and before any text-stream work queued after the flush (BERT's forward)."""
    from ctclip_mi355x import streams
    dev = torch.device('cuda', torch.cuda.current_device())
    ts = streams.text_stream(dev)
    if ts is None:
        pytest.skip('text stream disabled')
    main = torch.cuda.current_stream(dev)
    a = torch.randn(4096, 4096, device=dev)
    x = torch.zeros(1, device=dev)
    y = torch.zeros(1, device=dev)
    for _ in range(20):                       # long main-stream work ending in x = 1
        a = a @ a / 64
    x.fill_(1.0)
    streams.defer_text(dev, lambda: y.copy_(x * 2))
    x2 = torch.full((1,), 5.0, device=dev)
    for _ in range(10):
        a = a @ a / 64
    streams.mark_image_head(dev, streams.MARK_SITE)   # the deferred work may start after this point
    streams.flush_text(dev)
    with torch.cuda.stream(ts):
        z = y + x2                            # queued after the flush: sees the deferred result
    main.wait_stream(ts)
    torch.cuda.synchronize()
    assert y.item() == 2.0 and z.item() == 7.0


def test_eval_lean_forward_matches_full_forward():
    """The eval-mode lean 3D-ViT forward (round 6: under no_grad ViTLayerFn writes none of the
    backward-only tensors -- bf16 shadows, the LSE, FF1's h, the bf16 O) computes the same tokens as
    the full forward: encode_pooled under no_grad and with autograd recording, eval mode both,
    bit-identical pooled latents and VQ indices (grid 8 x 8 x 4 with the LN1 fold and fp16 operands,
    as the base config takes them)."""
    cfg = cfg_small()
    torch.manual_seed(0)
    model = build(cfg)
    model.eval()
    vt = model.visual_transformer
    hu = W.make_hu(2, cfg.vit).cuda()
    with torch.no_grad():
        p0, pb0 = vt.encode_pooled(hu)
        i0 = vt.vq.state.last_indices.clone()
    with torch.enable_grad():
        p1, pb1 = vt.encode_pooled(hu)
        i1 = vt.vq.state.last_indices.clone()
    assert p1.requires_grad                     # the full path (tensors saved for a backward)
    torch.cuda.synchronize()
    assert torch.equal(i0, i1)
    assert torch.equal(p0, p1.detach()) and torch.equal(pb0, pb1)
