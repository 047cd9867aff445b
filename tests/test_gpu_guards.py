"""Fail-loud guards of the 16-bit image-tower forward (round 6; VERDICT r05 Missing 3 / What's weak 2).

The reference computes the step in fp32 (ct_clip/CTCLIPTrainer.py:342,345-353), where a NaN / inf
simply propagates into every parameter.  This build stores fp16 / bf16 copies of activations, so:

* every fp16 producer checks its range (|v| <= 65504, finite) and ORs CT_STATUS_F16_RANGE into the
  sticky step status word; the VQ select flags tokens without a finite score (CT_STATUS_VQ_NONFINITE);
  the gradient-norm kernel flags a non-finite norm (CT_STATUS_NONFINITE_GRAD) into the Adam skip word;
* the trainer's Adam kernels skip a flagged step on every rank (parameters, moments untouched,
  gradients cleared), the guarded codebook EMA drops it, and the host raises NonFiniteStepError;
* trained-weight statistics: two layers on a residual stream with a large mean and outlier channels,
  the LN1 fold + fp16 forward against fp32 torch (oracle.transformer_forward), bound stated below."""
import math
import types

import pytest
import torch

from oracle import ctclip_oracle as O
from oracle import weights as W

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.fixture(scope='module')
def K():
    from ctclip_mi355x import kernels
    return kernels


def test_nonfinite_step_is_skipped_and_raises(K):
    """A NaN voxel in the (f32, [-1, 1]) input volume: its patch row goes NaN, the PEG's fp16 copy flags
    it, the VQ flags the token, the gradient norm is NaN.  The step is applied by nobody: parameters,
    Adam moments and the codebook stay bit-identical, the host raises NonFiniteStepError, and after
    reset_ln_status() the next step trains normally."""
    from test_gpu_model import build, cfg_small
    from ctclip_mi355x.trainer import CTClipTrainer, NonFiniteStepError
    cfg = cfg_small()
    torch.manual_seed(0)
    model = build(cfg)
    hu = W.make_hu(2, cfg.vit)
    ids, mask = W.make_text(2, 32, cfg.bert.vocab_size, ragged=True)
    text = types.SimpleNamespace(input_ids=ids.cuda(), attention_mask=mask.cuda())
    video = O.normalize_hu(hu).cuda()
    bad = video.clone()
    bad[1, 0, 17, 33, 71] = float('nan')
    K.reset_ln_status()
    tr = CTClipTrainer(model, lr=1e-3)
    tr.train_step(text, video)                      # one good step first (moments non-zero)
    tr.check()
    cbk = model.visual_transformer.vq._codebook
    snap = (tr.flat.data.clone(), tr.m.clone(), tr.v.clone(), cbk.embed.clone(), cbk.cluster_size.clone())
    tr.train_step(text, bad)
    with pytest.raises(NonFiniteStepError) as ei:
        tr.check()
    torch.cuda.synchronize()
    print('flagged step:', ei.value, 'bits', ei.value.bits)
    assert ei.value.bits & 4 and ei.value.bits & (2 | 8)
    for a, b, n in zip(snap, (tr.flat.data, tr.m, tr.v, cbk.embed, cbk.cluster_size),
                       ('params', 'adam m', 'adam v', 'codebook', 'cluster size')):
        assert torch.equal(a, b), n
    assert tr.flat.grad[:tr.flat.numel].abs().max().item() == 0.0      # cleared, not leaked forward
    K.reset_ln_status()
    loss = tr.train_step(text, video)
    tr.check()
    assert torch.isfinite(loss) and not torch.equal(snap[0], tr.flat.data)


def test_fp16_range_flag_in_layer(K):
    """A residual stream beyond fp16's range (|x| ~ 1e5) entering a 16-bit layer: the PEG's fp16 copy
    sets CT_STATUS_F16_RANGE (the f32 master and the bf16 copy are unaffected)."""
    from ctclip_mi355x import attention as A, functional as Fn
    torch.manual_seed(7)
    tr = A.Transformer(512, depth=1, dim_head=32, heads=8).cuda()
    geo = Fn.Geo(B=1, T=24, Hg=24, Wg=24, heads=8, dim_head=32, mode=0)
    xf = torch.randn(geo.M, 512, device='cuda')
    xf[5, 7] = 1e5
    K.reset_ln_status()
    prev = Fn.set_vit_f16(True)
    try:
        with torch.no_grad(), K.ln_guard():
            tr.run(xf, xf.bfloat16(), geo)
    finally:
        Fn.set_vit_f16(prev)
    torch.cuda.synchronize()
    assert K.ln_fused_status() & 2
    K.reset_ln_status()


@pytest.mark.parametrize('mode', [0, 1])
def test_trained_statistics_fold_fp16(K, mode):
    """Two layers on the 24^3 grid with a residual stream of mean +30, or with four outlier
    channels at 200x (the statistics a trained CT-CLIP_v2 stream may have): the default forward (LN1
    folded into the Q | K | V GEMM on fp16 operands) against fp32 torch, on the residual BRANCH
    (output - input, the PEG convs zeroed so the branch is attention + FeedForward).  Printed beside it: the same layers
    on a plain N(0, 1) stream and with the fold off (LayerNorm then Q on bf16 operands), and the
    split-fp16 x3 forward.  Stated bound: the fold's branch error on the shifted stream stays within
    4x its error on the plain stream and below 2e-2."""
    from ctclip_mi355x import attention as A, functional as Fn, precise
    torch.manual_seed(8)
    tr = A.Transformer(512, depth=2, dim_head=32, heads=8).cuda()
    with torch.no_grad():
        for n, p in tr.named_parameters():
            p.add_(0.02 * torch.randn_like(p))
            if 'dsconv' in n:
                p.zero_()     # PEG(x) = x: the branch below is attention + FeedForward only (an f32 conv of
                #               the shifted stream would otherwise dominate it and hide the fold's error)
    geo = Fn.Geo(B=1, T=24, Hg=24, Wg=24, heads=8, dim_head=32, mode=mode)
    sd = {k: v.detach() for k, v in tr.state_dict().items()}
    shape = (1, 24, 24, 24)

    def ref_fwd(x):
        # the two layers of oracle.transformer_forward without norm_out (it would normalise the
        # +30 / outlier stream away and dilute the branch)
        if mode == 1:
            x = x.view(1, 24, 24, 24, 512).permute(0, 2, 3, 1, 4).reshape(576, 24, 512)
        else:
            x = x.view(24, 576, 512)
        for i in range(2):
            lp = f'layers.{i}.'
            x = O.peg_forward(sd, lp + '0.', x, shape) + x
            x = O.attention_forward(sd, lp + '1.', x, 8, 32, None) + x
            x = O.ff_forward(sd, lp + '3.', x) + x
        if mode == 1:
            return x.reshape(1, 24, 24, 24, 512).permute(0, 3, 1, 2, 4).reshape(-1, 512)
        return x.reshape(-1, 512)

    def hip_fwd(x):
        xf, xb = x, x.bfloat16()
        for peg, attn, _, ff in tr.layers:
            xf, xb = Fn.ViTLayerFn.apply(xf, xb, None, geo, peg.dsconv.weight, peg.dsconv.bias, attn.norm.gamma,
                                         attn.q_scale, attn.k_scale, attn.to_q.weight, attn.to_kv.weight,
                                         attn.to_out.weight, ff[0].weight, ff[0].bias, ff[1].weight, ff[4].weight)
        return xf

    plain = torch.randn(geo.M, 512, device='cuda')
    mean30 = plain + 30.0
    outl = plain.clone()
    outl[:, [3, 100, 257, 400]] *= 200.0
    res = {}
    for name, x in (('plain', plain), ('mean30', mean30), ('outliers', outl)):
        ref = ref_fwd(x)
        for variant in ('fold_f16', 'unfold_bf16', 'split'):
            old_f16, old_fold = Fn.set_vit_f16(variant == 'fold_f16'), Fn._LN1_FOLD
            Fn._LN1_FOLD = variant == 'fold_f16'
            try:
                with torch.no_grad(), K.ln_guard(), precise.vit_precision_scope('split' if variant == 'split' else 'bf16'):
                    y = hip_fwd(x)
            finally:
                Fn.set_vit_f16(old_f16)
                Fn._LN1_FOLD = old_fold
            torch.cuda.synchronize()
            res[(name, variant)] = _rel(y - x, ref - x)
    for k, v in res.items():
        print(f'mode {mode} {k[0]:8s} {k[1]:12s}: residual-branch rel err vs fp32 {v:.2e}')
    assert K.ln_fused_status() == 0                 # in range: no flag
    for name in ('mean30', 'outliers'):
        assert res[(name, 'fold_f16')] < 2e-2
        assert res[(name, 'fold_f16')] < 4 * res[('plain', 'fold_f16')]
        assert res[(name, 'split')] < 1e-4
    assert all(math.isfinite(v) for v in res.values())
