"""configs[1] at full size on the GPU: the base CT-CLIP (480x480x240 volumes -> 24^3 tokens, 4+4
ViT layers, VQ 8192, BERT-base at 128 tokens) against the reference's OWN base-config output,
tests/golden/golden_base_b2.safetensors (tests/golden/make_golden.py --base ran
ct_clip/ct_clip.py:614-901 and ct_clip/ctvit.py:377-436 on these inputs and weights).

* stage checks: patch-embed / spatial / temporal head rows and per-volume token sums, CPB rows;
* the SURVEY 8(c) vector-quantiser contract, split in two:
  - the VQ op itself (bf16 MFMA candidates + f32 re-score, vq.hip) on the oracle's own f32
    pre-VQ tokens must return the oracle's argmax everywhere except f32-level ties (top-2 cosine
    margin < 1e-6);
  - end to end, every index the free-running HIP path picks differently from the reference must
    be explained by that token's own pre-VQ error: the oracle's score gap between its winner and
    the HIP choice is at most 2 * |l2norm(z_hip) - l2norm(z_oracle)| (both scores move by at most
    that much, Cauchy-Schwarz with unit codes).  Counts above / below the 1e-6 margin are printed;
* loss free-running against the fixture, logits / loss with the oracle forced onto the HIP indices
  (< 1e-3, the north-star bf16 tolerance); latents and free-running logits reported with their
  measured bounds;
* B = 8 (the bench workload) through train_step: finite, loss ~ ln 8 at init, weights move.
The oracle (fp32 CPU) runs the B = 2 forward here; it is pinned to the same fixture by
tests/test_oracle_golden.py::test_base_b2_matches_reference."""
import math
import os
import time  # noqa: F401
import types

import pytest
import torch
import torch.nn.functional as F

from oracle import ctclip_oracle as O
from oracle import weights as W

pytestmark = pytest.mark.gpu

CFG = O.BASE
HERE = os.path.dirname(os.path.abspath(__file__))


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.fixture(scope='module')
def base():
    from safetensors.torch import load_file
    from test_gpu_model import build
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    g = load_file(os.path.join(HERE, 'golden', 'golden_base_b2.safetensors'))
    sd = W.make_state_dict(CFG)
    model = build(CFG)
    hu = W.make_hu(2, CFG.vit)
    ids, mask = W.make_text(2, 128, CFG.bert.vocab_size)
    trace = {}
    with torch.no_grad():
        ref = O.ctclip_forward(sd, ids, mask, O.normalize_hu(hu), CFG, training=False, trace=trace)
    text = types.SimpleNamespace(input_ids=ids.cuda(), attention_mask=mask.cuda())
    return dict(g=g, sd=sd, model=model, hu=hu, ids=ids, mask=mask, text=text, ref=ref, trace=trace)


def test_oracle_full_size_matches_fixture(base):
    """The checker itself at full size: the oracle's indices / latents / loss vs the reference's."""
    g, ref = base['g'], base['ref']
    mism = (ref['indices'].reshape(-1).to(torch.int32) != g['out.vq_indices'].reshape(-1)).sum().item()
    print('oracle vs reference VQ index mismatches:', mism, 'of', g['out.vq_indices'].numel())
    assert mism <= 3
    assert (ref['text_latents'] - g['out.text_latents']).abs().max().item() < 1e-4
    assert abs(ref['loss'].item() - g['out.loss'].item()) < 1e-4


def test_stages_full_size(base):
    g, model = base['g'], base['model']
    vt = model.visual_transformer
    model.eval()
    tr = {}
    with torch.no_grad():
        zf, zb, geo = vt.encode_tokens(base['hu'].cuda(), trace=tr)
        cpb = vt.spatial_rel_pos_bias.dense(24, 24)
    torch.cuda.synchronize()
    D = CFG.vit.dim
    pe, sp = tr['patch_emb'], tr['spatial_out']
    # temporal head rows are in the reference's '(b h w) t d' order: row r = (hw = r // 24, t = r % 24)
    r = torch.arange(256)
    trow = (r % 24) * 576 + r // 24
    checks = {
        'patch_emb_head': (pe[:256], g['out.patch_emb_head'], 1e-2),
        'patch_emb_sum': (pe.view(2, -1, D).double().sum(1), g['out.patch_emb_sum'], 1e-2),
        'spatial_out_head': (sp[:256], g['out.spatial_out_head'], 2e-2),
        'temporal_out_head': (zf[trow.cuda()], g['out.temporal_out_head'], 3e-2),
        'temporal_out_sum': (zf.view(2, -1, D).double().sum(1), g['out.temporal_out_sum'], 3e-2),
        'cpb_rows': (cpb[:, :4, :], g['out.cpb_rows'], 1e-5),
    }
    bad = []
    for k, (a, b, tol) in checks.items():
        e = rel(a, b)
        print(f'{k}: rel err {e:.3e} (tol {tol})')
        if not e < tol:
            bad.append((k, e))
    assert not bad, bad
    # the patch / token index maps are exact: the f32 [-1, 1] video takes the int16 path bit-for-bit
    with torch.no_grad():
        tr2 = {}
        vt.encode_tokens(O.normalize_hu(base['hu']).cuda(), trace=tr2)
    assert torch.equal(tr2['patch_emb'], pe)
    base['zf'], base['zb'] = zf, zb
    model.train()


def _oracle_tokens(base):
    t = base['trace']['temporal_out']                  # (b, t, h, w, d) = canonical HIP row order
    return t.reshape(-1, CFG.vit.dim).contiguous()


def test_vq_op_exact_on_oracle_tokens(base):
    """SURVEY 8(c) for the quantiser op: same f32 tokens in -> the oracle's argmax out, except
    f32 ties (top-2 margin < 1e-6)."""
    from ctclip_mi355x import functional as Fn
    from ctclip_mi355x import kernels as K
    vt = base['model'].visual_transformer
    zo = _oracle_tokens(base)
    cb = vt.vq._codebook.embed.view(-1, CFG.vit.dim)
    with torch.no_grad():
        zf = zo.cuda()
        idx, _ = Fn.vq_assign(zf, K.cast_bf16(zf), cb, vt.vq.state)
    torch.cuda.synchronize()
    so = F.normalize(zo, dim=-1) @ base['sd']['visual_transformer.vq._codebook.embed'][0].t()
    top2 = so.topk(2, dim=1)
    oi = top2.indices[:, 0]
    margin = top2.values[:, 0] - top2.values[:, 1]
    diff = idx.cpu().long() != oi
    print(f'VQ op on oracle tokens: {diff.sum().item()} mismatches of {diff.numel()}; '
          f'{(margin < 1e-6).sum().item()} oracle rows with top-2 margin < 1e-6; '
          f'min margin {margin.min().item():.3e}')
    assert (diff & (margin >= 1e-6)).sum().item() == 0


def test_vq_free_running_contract(base):
    """End to end: every HIP index that differs from the reference's is a near-tie explained by
    that token's measured pre-VQ error (see module docstring)."""
    g, sd = base['g'], base['sd']
    if 'zf' not in base:
        pytest.skip('needs test_stages_full_size')
    from ctclip_mi355x import functional as Fn
    vt = base['model'].visual_transformer
    cb = vt.vq._codebook.embed.view(-1, CFG.vit.dim)
    with torch.no_grad():
        idx, _ = Fn.vq_assign(base['zf'], base['zb'], cb, vt.vq.state)
    idx = idx.cpu().long()
    gi = g['out.vq_indices'].reshape(-1).long()
    diff = (idx != gi).nonzero().flatten()
    zo = _oracle_tokens(base)
    xo = F.normalize(zo[diff], dim=-1)
    xh = F.normalize(base['zf'][diff.cuda()].cpu(), dim=-1)
    E = sd['visual_transformer.vq._codebook.embed'][0]
    so = xo @ E.t()
    gap = so.gather(1, gi[diff][:, None]).squeeze(1) - so.gather(1, idx[diff][:, None]).squeeze(1)
    bound = 2 * (xh - xo).norm(dim=1)
    tok_err = (F.normalize(base['zf'].cpu(), dim=-1) - F.normalize(zo, dim=-1)).norm(dim=1)
    n = gi.numel()
    print(f'free-running VQ: {diff.numel()} of {n} indices differ ({100 * diff.numel() / n:.2f} %); '
          f'oracle margin < 1e-6: {(gap < 1e-6).sum().item()}, above: {(gap >= 1e-6).sum().item()}; '
          f'max gap {gap.max().item() if diff.numel() else 0:.3e}; '
          f'pre-VQ |dxn| median {tok_err.median().item():.3e} max {tok_err.max().item():.3e}')
    unexplained = (gap > bound + 1e-6).sum().item()
    assert unexplained == 0, unexplained
    # round 5 (fp16 forward GEMMs + f32-tap PEG): 250 of 27,648 above the 1e-6 margin
    # (667 with the all-bf16 tower of round 4); pre-VQ |dxn| median 4.6e-3 (1.07e-2)
    assert (gap >= 1e-6).sum().item() < 400
    assert diff.numel() < 0.02 * n


def test_latents_and_loss_full_size(base):
    g, sd, model, text = base['g'], base['sd'], base['model'], base['text']
    model.eval()
    with torch.no_grad():
        _, _, t_raw, i_raw = model.encode(text, base['hu'].cuda())
        idx = model.visual_transformer.vq.state.last_indices.cpu()
        loss = model(text, base['hu'].cuda(), return_loss=True)
    torch.cuda.synchronize()
    tl, il = F.normalize(t_raw, dim=-1).cpu(), F.normalize(i_raw, dim=-1).cpu()
    e = math.e            # temperature.exp() at init (ct_clip.py:568,796)
    logits = tl @ il.t() * e
    g_logits = g['out.text_latents'] @ g['out.image_latents'].t() * e
    dt = (tl - g['out.text_latents']).abs().max().item()
    di = (il - g['out.image_latents']).abs().max().item()
    dlog = (logits - g_logits).abs().max().item()
    dl = abs(loss.item() - g['out.loss'].item())
    print(f'free-running vs reference fixture: text latents {dt:.2e}, image latents {di:.2e}, logits {dlog:.2e}, '
          f'loss {loss.item():.6f} vs {g["out.loss"].item():.6f} (|d| {dl:.2e})')
    # text latents: 12 BERT-base layers on split hi / lo weights (bf16 activations) -- the north-star
    # 1e-3 (single bf16 weights gave 1.4e-3, tools/bert_precision.py); the loss within 1e-3
    # free-running (6.2e-4 measured); the image latents / logits of the DEFAULT bf16 image tower carry
    # its ~2 % near-tie VQ flips (2.5e-2 / 5.3e-2 measured): a flipped token swaps in a different
    # codebook row, so they meet 1e-3 once the indices agree (forced, below) or in the f32 image
    # mode (test_f32_image_mode_vq_contract)
    assert dt < 1e-3
    # free-running loss: every VQ index that flips on a near-tie swaps a codebook row into the pooled
    # latent, so |dloss| scales with the flip count.  Round 5's fp16 forward GEMMs + f32-tap PEG cut
    # the pre-VQ error 1.07e-2 -> 4.6e-3 and the flips 667 -> 250 (0.9 %): loss |d| 4.7e-4 measured
    # (round 4's all-bf16 tower: 1.9e-3).  The north-star 1e-3, free-running:
    assert dl < 1e-3
    assert di < 0.04 and dlog < 0.04
    with torch.no_grad():
        forced = O.ctclip_forward(sd, base['ids'], base['mask'], O.normalize_hu(base['hu']), CFG,
                                  training=False, force_ind=idx)
    fi = (il - forced['image_latents']).abs().max().item()
    f_logits = forced['text_latents'] @ forced['image_latents'].t() * e
    flog = (logits - f_logits).abs().max().item()
    fl = abs(loss.item() - forced['loss'].item())
    print(f'oracle forced onto the HIP indices: image latents {fi:.2e}, logits {flog:.2e}, loss |d| {fl:.2e}')
    assert fi < 1e-3
    assert fl < 1e-3
    # logits = e * text . image within the north-star 1e-3 (1.18e-3 before the split weights)
    assert flog < 1e-3
    model.train()


def _time_encode(model, hu, reps=3):
    """ms per CTCLIP image-tower forward (encode_pooled + projection) under no_grad, HIP events."""
    vt = model.visual_transformer
    W = model.to_visual_latent.weight
    with torch.no_grad():
        model._project(W, model._visual_weight_bf16(W), *vt.encode_pooled(hu))   # warm
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            model._project(W, model._visual_weight_bf16(W), *vt.encode_pooled(hu))
        e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


@pytest.mark.parametrize('mode', ['f32', 'split'])
def test_f32_image_mode_vq_contract(base, mode):
    """SURVEY 8(c) LITERALLY, in the opt-in precise image towers (precise.py: 'f32' = f32 MFMA GEMMs,
    'split' = split-fp16 x3 GEMMs, round 6): free-running at configs[1] size against the reference's
    own output (golden_base_b2), every VQ index equals the reference's except where the oracle's fp32
    top-2 cosine margin is below 1e-6; image latents, logits and loss within the north-star 1e-3.  Also
    reports the tower's forward cost against the default tower."""
    from ctclip_mi355x import precise
    g, sd, model, text = base['g'], base['sd'], base['model'], base['text']
    hu = base['hu'].cuda()
    model.eval()
    old = precise.set_vit_precision(mode)
    try:
        with torch.no_grad():
            tr = {}
            zf, _, _ = model.visual_transformer.encode_tokens(hu, trace=tr)
            _, _, t_raw, i_raw = model.encode(text, hu)
            idx = model.visual_transformer.vq.state.last_indices.cpu().long()
            loss = model(text, hu, return_loss=True)
        torch.cuda.synchronize()
        ms_f32 = _time_encode(model, hu)
    finally:
        precise.set_vit_precision(old)
    ms_bf16 = _time_encode(model, hu)
    zo = _oracle_tokens(base)
    tok = rel(zf, zo)
    E = sd['visual_transformer.vq._codebook.embed'][0]
    so = F.normalize(zo, dim=-1) @ E.t()
    top2 = so.topk(2, dim=1)
    margin = top2.values[:, 0] - top2.values[:, 1]
    gi = g['out.vq_indices'].reshape(-1).long()
    diff = idx != gi
    above = (diff & (margin >= 1e-6)).sum().item()
    tl, il = F.normalize(t_raw, dim=-1).cpu(), F.normalize(i_raw, dim=-1).cpu()
    e = math.e
    dlog = (tl @ il.t() * e - g['out.text_latents'] @ g['out.image_latents'].t() * e).abs().max().item()
    di = (il - g['out.image_latents']).abs().max().item()
    dl = abs(loss.item() - g['out.loss'].item())
    # the remaining index differences are f32 ties (margin < 1e-6: the oracle and the reference,
    # both fp32 CPU, split on them too -- test_oracle_full_size_matches_fixture); a tie swaps one
    # codebook row into the pooled latent, so latents / logits are compared with the oracle on the
    # same indices (ties resolved alike)
    with torch.no_grad():
        forced = O.ctclip_forward(sd, base['ids'], base['mask'], O.normalize_hu(base['hu']), CFG,
                                  training=False, force_ind=idx.to(torch.int32))
    fi = (il - forced['image_latents']).abs().max().item()
    flog = (tl @ il.t() * e - forced['text_latents'] @ forced['image_latents'].t() * e).abs().max().item()
    fl = abs(loss.item() - forced['loss'].item())
    print(f'{mode} image tower: pre-VQ tokens rel {tok:.2e} vs oracle; VQ {diff.sum().item()} of {gi.numel()} '
          f'differ from the reference ({above} with oracle margin >= 1e-6); free-running vs the reference: image '
          f'latents {di:.2e}, logits {dlog:.2e}, loss |d| {dl:.2e}; vs the oracle on the same indices: image '
          f'latents {fi:.2e}, logits {flog:.2e}, loss |d| {fl:.2e}; image-tower forward at B=2: {mode} '
          f'{ms_f32:.1f} ms vs default {ms_bf16:.1f} ms')
    assert above == 0
    assert dl < 1e-3                  # free-running, the north-star loss tolerance
    assert dlog < 5e-3                # free-running logits: only f32 ties (margin < 1e-6) can flip
    if mode == 'split':
        # the split tower (round 6) also resolves the f32 tie as the reference does: the literal
        # north-star logits bound free-running (4.5e-4 measured)
        assert dlog < 1e-3 and di < 1e-3
    assert fi < 1e-4 and flog < 1e-3 and fl < 1e-3
    model.train()


@pytest.mark.parametrize('mode', ['f32', 'split'])
def test_f32_mode_forward_backward_full_size(base, mode):
    """The trainable f32 mode at configs[1] size (B = 2, train mode, autograd through the tower):
    the loss the step differentiates meets the north-star 1e-3 against the reference's output
    free-running, every VQ index agrees with the reference's except f32 ties (margin < 1e-6), and
    the (bf16) backward produces finite gradients for both towers.  Reports the f32-mode forward +
    backward time against the default mode's."""
    from ctclip_mi355x import precise
    g, sd, model, text = base['g'], base['sd'], base['model'], base['text']
    hu = base['hu'].cuda()
    cbk = model.visual_transformer.vq._codebook
    saved = cbk.embed.clone(), cbk.cluster_size.clone()
    model.train()

    def fwd_bwd():
        model.zero_grad(set_to_none=True)
        loss = model(text, hu, return_loss=True)
        loss.backward()
        return loss

    try:
        times = {}
        for md in ('bf16', mode, mode):          # second run of the mode: warm timing
            with precise.vit_precision_scope(md):
                with torch.no_grad():
                    cbk.embed.copy_(saved[0])
                    cbk.cluster_size.copy_(saved[1])
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                loss = fwd_bwd()
                e.record()
                torch.cuda.synchronize()
                times[md] = s.elapsed_time(e)
        idx = model.visual_transformer.vq.state.last_indices.cpu().long()
        p_img = model.visual_transformer.enc_spatial_transformer.layers[0][1].to_q.weight
        p_txt = model.text_transformer.encoder.layer[11].output.dense.weight
        gi_img, gi_txt = p_img.grad.norm().item(), p_txt.grad.norm().item()
    finally:
        with torch.no_grad():
            cbk.embed.copy_(saved[0])
            cbk.cluster_size.copy_(saved[1])
        model.zero_grad(set_to_none=True)
    zo = _oracle_tokens(base)
    E = sd['visual_transformer.vq._codebook.embed'][0]
    so = F.normalize(zo, dim=-1) @ E.t()
    top2 = so.topk(2, dim=1)
    margin = top2.values[:, 0] - top2.values[:, 1]
    gi = g['out.vq_indices'].reshape(-1).long()
    diff = idx != gi
    above = (diff & (margin >= 1e-6)).sum().item()
    dl = abs(loss.item() - g['out.loss'].item())
    print(f'{mode} mode, train-mode forward + backward at B=2: loss {loss.item():.6f} vs reference '
          f'{g["out.loss"].item():.6f} (|d| {dl:.2e}); VQ {diff.sum().item()} of {gi.numel()} differ '
          f'({above} above the 1e-6 margin); grad norms image {gi_img:.3e} text {gi_txt:.3e}; '
          f'fwd+bwd ms: default {times["bf16"]:.1f}, {mode} {times[mode]:.1f}')
    assert above == 0
    assert dl < 1e-3
    assert math.isfinite(gi_img) and gi_img > 0 and math.isfinite(gi_txt) and gi_txt > 0


def test_train_step_batch8_full_size(base):
    """configs[1] itself (B = 8): one full train step -- finite loss near ln 8 at init, finite
    non-zero gradient norm, parameters of both towers updated."""
    from ctclip_mi355x.trainer import CTClipTrainer
    model = base['model']
    for k in ('zf', 'zb'):
        base.pop(k, None)
    dev = torch.device('cuda')
    gen = torch.Generator(device=dev).manual_seed(1234)
    hu = torch.randint(-1200, 1201, (8, 1, 240, 480, 480), generator=gen, device=dev,
                       dtype=torch.int32).to(torch.int16)
    ids = torch.randint(5, CFG.bert.vocab_size, (8, 128), generator=gen, device=dev)
    ids[:, 0], ids[:, -1] = 2, 3
    text = types.SimpleNamespace(input_ids=ids, attention_mask=torch.ones_like(ids))
    model.train()
    tr = CTClipTrainer(model)
    p_img = model.visual_transformer.enc_temporal_transformer.layers[3][3][1].weight
    p_txt = model.text_transformer.encoder.layer[11].output.dense.weight
    b_img, b_txt = p_img.detach().clone(), p_txt.detach().clone()
    loss = tr.train_step(text, hu)
    torch.cuda.synchronize()
    print(f'B=8 full-size train step: loss {loss.item():.5f} (ln 8 = {math.log(8):.5f}), '
          f'grad norm {tr.norm[0].item():.4e}')
    assert torch.isfinite(loss) and abs(loss.item() - math.log(8)) < 0.1
    assert math.isfinite(tr.norm[0].item()) and tr.norm[0].item() > 0
    assert not torch.equal(b_img, p_img.detach()) and not torch.equal(b_txt, p_txt.detach())
    assert model.visual_transformer.vq.state.last_indices.numel() == 8 * 24 ** 3
