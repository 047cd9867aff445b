"""The split-fp16 "x3" image tower (precise.set_vit_precision('split'), round 6): operands as fp16
(hi, lo) image pairs (~22 mantissa bits), three fp16 MFMA products per K-step (Ah Bh + Ah Bl + Al Bh)
into one f32 accumulator on the 8-phase GEMM (gemm256.hip, ctclip_gemm_args.A_lo / B_lo).

* the split producers: ctclip_split_f16 / ctclip_pack_rows_x3 (range flag into the step status word),
  the patch LayerNorm, the LayerNorm and the f32-tap PEG with their lo outputs -- hi + lo equals the
  f32 value to 2^-22 relative;
* the x3 GEMM against an f64 matmul of the ORIGINAL f32 operands: relative 2e-6 (the bf16 / fp16
  GEMMs are at 1e-3 / 2e-4; the f32 GEMM ctclip_sgemm_tn at ~5e-7 against the same reference), f32 rows
  with bias / residual / bf16 copy, and the GEGLU pair epilogue (h fp16, g as an fp16 pair and bf16);
* the whole tower at base widths on the reduced volume against the fp32 oracle: pre-VQ tokens at the
  f32 level, VQ indices identical except oracle near-ties (the configs[1]-size contract is in
  test_gpu_base.py)."""
import pytest
import torch
import torch.nn.functional as F

from oracle import ctclip_oracle as O
from test_gpu_ops import _peg_ref, rel

pytestmark = pytest.mark.gpu
dev = 'cuda'


@pytest.fixture(scope='module')
def K():
    from ctclip_mi355x import kernels
    return kernels


def _pair(hi, lo):
    return hi.double() + lo.double()


def _status(K):
    return int(K.status_word(torch.device(dev)).item())


def test_split_f16_pair_and_range_flag(K):
    torch.manual_seed(11)
    x = torch.randn(1000, 520, device=dev) * torch.logspace(-3, 3, 520, device=dev)
    hi, lo = K.split_f16(x)
    torch.cuda.synchronize()
    assert torch.equal(hi, x.half())
    err = (_pair(hi, lo) - x.double()).abs()
    # 2^-22 relative (lo normal) or the fp16 subnormal step of lo (2^-25 absolute)
    assert (err <= x.double().abs() * 2.0 ** -22 + 2.0 ** -25).all()
    K.reset_ln_status()
    assert _status(K) == 0
    bad = x.clone()
    bad[7, 3] = 1e6
    K.split_f16(bad)
    assert _status(K) & 2
    K.reset_ln_status()
    bad[7, 3] = float('nan')
    K.split_f16(bad)
    assert _status(K) & 2
    K.reset_ln_status()
    # the scale: hi + lo of x * 16
    hi, lo = K.split_f16(x[:, :512].contiguous(), scale=16.0)
    assert ((_pair(hi, lo) / 16 - x[:, :512].double()).abs() <= x[:, :512].double().abs() * 2.0 ** -22 + 2.0 ** -29).all()
    assert _status(K) == 0


def test_pack_rows_x3(K):
    from ctclip_mi355x import functional as Fn
    torch.manual_seed(12)
    inner, D = 1365, 512
    W1 = torch.randn(2 * inner, D, device=dev) * 0.02
    cs = torch.rand(D, device=dev) + 0.5
    P = Fn.ff_pad(inner)
    rm = Fn.ff1_rowmap(inner, W1.device)
    hi, lo = K.pack_rows_x3(W1, 2 * P, D + 64, rowmap=rm, colscale=cs)
    ref = K.pack_rows_f32(W1, 2 * P, D + 64, rowmap=rm, colscale=cs).double() * K.X3_WSCALE
    # 2^-22 relative, or lo's fp16 subnormal step (2^-25 absolute) for the smallest entries
    assert ((_pair(hi, lo) - ref).abs() <= ref.abs() * 2.0 ** -22 + 2.0 ** -25).all()
    assert hi[:, D:].abs().max().item() == 0 and lo[rm.cpu() < 0].abs().max().item() == 0
    assert _status(K) == 0


def _x3_operands(K, M, N, Kd, seed=13):
    torch.manual_seed(seed)
    x = torch.randn(M, Kd, device=dev)
    w = torch.randn(N, Kd, device=dev) / Kd ** 0.5
    return x, w, K.split_f16(x), K.pack_rows_x3(w, N, Kd)


@pytest.mark.parametrize('M,N,Kd', [(300, 256, 512), (8192, 768, 512), (4096, 512, 1408), (2500, 512, 4032)])
def test_x3_gemm_f32_rows(K, M, N, Kd):
    x, w, xs, ws = _x3_operands(K, M, N, Kd)
    b = torch.randn(N, device=dev)
    r = torch.randn(M, N, device=dev)
    ref = x.double() @ w.double().t()
    y, yb = K.linear_x3(xs, ws, want_bf16=True)
    torch.cuda.synchronize()
    e = rel(y, ref)
    e32 = rel(K.linear_f32(x, w)[0], ref)
    e16 = rel(K.linear(x.half(), w.half(), out_dtype=torch.float32), ref)
    print(f'x3 GEMM {M}x{N}x{Kd}: rel {e:.2e} (f32 MFMA GEMM {e32:.2e}, fp16 GEMM {e16:.2e})')
    assert e < 2e-6
    assert torch.equal(yb, y.bfloat16())
    y2, _ = K.linear_x3(xs, ws, bias=b, residual=r)
    assert rel(y2, ref + b.double() + r.double()) < 2e-6


def test_x3_gemm_geglu(K):
    """FF1 + GEGLU on the x3 GEMM: h (fp16) in the derivative form [gelu(gate) | x gelu'(gate)] of
    the x3 product (round 6: the GEGLU backward's two factors); g = gelu(gate) x from the UNROUNDED
    f32 product, stored as an fp16 pair (hi + lo = g to 2^-22) and as bf16; padded columns 0."""
    from ctclip_mi355x import functional as Fn
    torch.manual_seed(14)
    M, D, inner = 4096, 512, 1365
    x = torch.randn(M, D, device=dev)
    W1 = torch.randn(2 * inner, D, device=dev) / D ** 0.5
    P = Fn.ff_pad(inner)
    rm = Fn.ff1_rowmap(inner, W1.device)
    h, (gh, gl), gb = K.linear_x3_geglu(K.split_f16(x), K.pack_rows_x3(W1, 2 * P, D, rowmap=rm))
    W1p = K.pack_rows_f32(W1, 2 * P, D, rowmap=rm).double()
    hf = x.double() @ W1p.t()
    hp = hf.view(M, P // 32, 2, 32)
    xp, gp = hp[:, :, 0], hp[:, :, 1]
    cdf = 0.5 * (1 + torch.erf(gp / 2 ** 0.5))
    pdf = torch.exp(-0.5 * gp * gp) / (2 * torch.pi) ** 0.5
    hd = torch.stack([F.gelu(gp), xp * (cdf + gp * pdf)], 2).reshape(M, 2 * P)
    assert rel(h, hd) < 5e-4                         # fp16 storage of the derivative form
    ref = (F.gelu(hp[:, :, 1]) * hp[:, :, 0]).reshape(M, P)
    g = _pair(gh, gl)
    e = rel(g, ref)
    print(f'x3 GEGLU: g rel {e:.2e}')
    assert e < 2e-6
    assert rel(gb, ref) < 5e-3
    assert g[:, inner:].abs().max().item() == 0.0


def test_x3_producers_lo_outputs(K):
    """The producers' lo images: the patch LayerNorm, the LayerNorm and the f32-tap PEG write
    fp16(v - fp16(v)) beside the fp16 copy, so hi + lo is their f32 output to 2^-22."""
    torch.manual_seed(15)
    x = torch.randn(3000, 512, device=dev) * 3 + 1
    g = torch.rand(512, device=dev) + 0.5
    b = torch.randn(512, device=dev) * 0.1
    yb, yf, m, r, (yh, yl) = K.layernorm_fwd(x, g, b, 1e-5, out_f32=True, out_x3=True)
    assert torch.equal(yh, yf.half())
    assert ((_pair(yh, yl) - yf.double()).abs() <= yf.double().abs() * 2.0 ** -22 + 2.0 ** -25).all()
    shape, D = (1, 24, 24, 24), 512
    M = 24 ** 3
    xp = torch.randn(M, D, device=dev)
    w = torch.randn(D, 1, 3, 3, 3, device=dev) * 0.2
    bb = torch.randn(D, device=dev) * 0.1
    for mode in (0, 1):
        of, ob, (oh, ol), _, _ = K.peg_fwd_x32(xp, *shape, w, bb, mode, want_x3=True)
        assert torch.equal(oh, of.half()) and torch.equal(ob, of.bfloat16())
        assert ((_pair(oh, ol) - of.double()).abs() <= of.double().abs() * 2.0 ** -22 + 2.0 ** -25).all()
        assert rel(of, _peg_ref(xp.double(), w.double(), bb.double(), shape, mode)) < 2e-7
    from oracle import weights as W
    from ctclip_mi355x.layers import patch_offsets
    vit = O.ViTConfig(dim=512, codebook_size=64, image_size=80, patch_size=20, temporal_patch_size=10,
                      spatial_depth=1, temporal_depth=1, dim_head=32, heads=8, frames=20)
    hu = W.make_hu(2, vit).to(dev)
    offs = patch_offsets(1, 10, 20, 20, 80, 80).to(dev)
    xb, (xh, xl) = K.patch_ln(hu, True, 10, 20, offs, ld=4032, want_x3=True)
    xf = K.patch_ln_f32(hu, True, 10, 20, offs, torch.ones(4000, device=dev), torch.zeros(4000, device=dev))
    assert torch.equal(xb, K.patch_ln(hu, True, 10, 20, offs, ld=4032))
    assert rel(_pair(xh, xl)[:, :4000], xf.double()) < 1e-6
    assert xh[:, 4000:].abs().max().item() == 0 and xl[:, 4000:].abs().max().item() == 0
    assert _status(K) == 0
    big = x * 1e5
    K.layernorm_fwd(big, g * 1e5, None, 1e-5, out_x3=True)
    assert _status(K) & 2
    K.reset_ln_status()


def test_split_tower_matches_oracle_small(K):
    """The split tower (base widths, 160 x 160 x 40 volume, 2 + 2 layers) against the fp32 oracle:
    pre-VQ tokens at the f32 level (as the f32 mode, test_gpu_f32path.py), VQ indices identical except
    oracle near-ties; and a train step in the mode moves the weights with finite loss."""
    import importlib.util
    import os
    import types
    spec = importlib.util.spec_from_file_location('tgm', os.path.join(os.path.dirname(__file__), 'test_gpu_model.py'))
    tgm = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(tgm)
    from oracle import weights as W
    from ctclip_mi355x import precise
    from ctclip_mi355x.trainer import CTClipTrainer
    cfg = tgm.cfg_small()
    model = tgm.build(cfg)
    sd = W.make_state_dict(cfg)
    hu = W.make_hu(2, cfg.vit)
    ids, mask = W.make_text(2, 32, cfg.bert.vocab_size, ragged=True)
    trace = {}
    with torch.no_grad():
        ref = O.ctclip_forward(sd, ids, mask, O.normalize_hu(hu), cfg, training=False, trace=trace)
    vt = model.visual_transformer
    model.eval()
    with precise.vit_precision_scope('split'):
        with torch.no_grad():
            zf, _, _ = vt.encode_tokens(hu.cuda())
            ids_h = vt(hu.cuda(), return_only_codebook_ids=True).reshape(-1).cpu()
        with precise.vit_precision_scope('f32'):
            with torch.no_grad():
                z32, _, _ = vt.encode_tokens(hu.cuda())
    zo = trace['temporal_out'].reshape(-1, cfg.vit.dim)
    r = rel(zf.cpu(), zo)
    r32 = rel(z32.cpu(), zo)
    E = sd['visual_transformer.vq._codebook.embed'][0]
    so = F.normalize(zo, dim=-1) @ E.t()
    top2 = so.topk(2, dim=1)
    margin = top2.values[:, 0] - top2.values[:, 1]
    diff = ids_h != ref['indices'].reshape(-1).cpu()
    print(f'split tower (small): tokens rel {r:.2e} (f32 mode {r32:.2e}), VQ diffs {diff.sum().item()} '
          f'({(diff & (margin >= 1e-6)).sum().item()} above the 1e-6 margin)')
    assert r < 1e-5
    assert (diff & (margin >= 1e-6)).sum().item() == 0
    assert _status(K) == 0
    text = types.SimpleNamespace(input_ids=ids.cuda(), attention_mask=mask.cuda())
    model.train()
    tr = CTClipTrainer(model, lr=1e-4)
    p = model.visual_transformer.enc_spatial_transformer.layers[0][3][1].weight
    before = p.detach().clone()
    with precise.vit_precision_scope('split'):
        l1 = tr.train_step(text, hu.cuda())
        l2 = tr.train_step(text, hu.cuda())
        tr.flush()
    assert torch.isfinite(l1) and torch.isfinite(l2) and not torch.equal(before, p.detach())


@pytest.mark.parametrize('case', ['spatial', 'spatial_5x7', 'temporal'])
def test_attention_x3(K, case):
    """The split-fp16 x3 attention forward (ctclip_attn_fwd_x3) against the f64 reference: O (hi + lo)
    at the f32 level, its bf16 copy the rounding of it, and the natural-log LSE the bf16 backward
    (ctclip_attn_bwd) reads."""
    from test_gpu_ops import _attn_ref, _cpb_table, _gather_rows
    torch.manual_seed(16)
    if case.startswith('spatial'):
        gh, gw = {'spatial': (24, 24), 'spatial_5x7': (5, 7)}[case]
        L, H, D, nseq = gh * gw, 8, 32, 3
        M, seq, grid = nseq * L, (1, L, 0, 1), (gh, gw)
        u, bins = _cpb_table(H, gh, gw)
        bias = u[:, bins].double()
    else:
        B, T, HW, H = 2, 24, 20, 8
        L, D, nseq = T, 32, B * HW
        M, seq, grid = B * T * HW, (HW, T * HW, 1, HW), (0, 0)
        u, bias = None, None
    rows = _gather_rows(*seq, nseq, L)
    q = F.normalize(torch.randn(M, H, D, device=dev), dim=-1).reshape(M, H * D)
    kv = torch.randn(M, 2 * H * D, device=dev)
    kv[:, :H * D] = F.normalize(kv[:, :H * D].reshape(M, H, D), dim=-1).reshape(M, H * D)
    k, v = kv[:, :H * D], kv[:, H * D:]
    (oh, ol), ob, lse = K.attn_fwd_x3(q, k, v, L=L, H=H, D=D, nseq=nseq, scale=8.0, seq=seq, bias_u=u, grid=grid)
    ref = _attn_ref(q.double(), k.double(), v.double(), rows, H, D, 8.0, bias)
    o = _pair(oh, ol)
    e = rel(o, ref)
    e32 = rel(K.attn_fwd_f32(q, k, v, L=L, H=H, D=D, nseq=nseq, scale=8.0, seq=seq, bias_u=u, grid=grid), ref)
    print(f'x3 attention {case}: O rel {e:.2e} (f32 kernel {e32:.2e})')
    assert e < 1e-6
    # the bf16 copy is the rounding of the kernel's f32 O: half an ulp (2^-8 relative just above a power
    # of two) plus that O's own absolute error, bounded here by twice the pair's worst element error
    eabs = (o - ref).abs().max().item()
    slack = ((ob.double() - ref).abs() - ref.abs() * 2.0 ** -8).max().item()
    print(f'  bf16 copy: max excess over half an ulp {slack:.2e} (pair max abs err {eabs:.2e})')
    assert slack <= 2 * eabs + 1e-9
    # LSE: ln sum_k exp(8 q.k + bias) per (head, query row)
    qd, kd = q.double().view(M, H, D), k.double().view(M, H, D)
    lref = torch.empty(H, M, dtype=torch.float64, device=dev)
    for s_ in range(nseq):
        r = rows[s_]
        sc = 8.0 * torch.einsum('ihd,jhd->hij', qd[r], kd[r])
        if bias is not None:
            sc = sc + bias
        lref[:, r] = torch.logsumexp(sc, dim=-1)
    assert (lse.double() - lref).abs().max().item() < 1e-5
