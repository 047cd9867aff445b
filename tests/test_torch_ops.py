"""torch.library custom ops (ctclip_mi355x/ops.py): registration, fake (meta)
shapes and CPU refusal here; numerics and gradients against torch fp32 references of the same op
on the GPU (the kernels behind them are the model's own, called through the C-ABI)."""
import math

import pytest
import torch
import torch.nn.functional as F
from torch._subclasses.fake_tensor import FakeTensorMode

from ctclip_mi355x import ops  # noqa: F401  (registers torch.ops.ctclip)

BF, F32 = torch.bfloat16, torch.float32
OPS = ('gemm_bf16', 'layernorm', 'cos_attn', 'clip_infonce', 'vq_cos_argmax', 'peg_dwconv3d', 'cpb_mlp',
       'patch_embed_i16', 'bert_layer')


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


# ------------------------------------------------------------------------------ host side
def test_ops_registered_with_fake_shapes():
    for n in OPS:
        assert hasattr(torch.ops.ctclip, n), n
    with FakeTensorMode():
        x = torch.empty(256, 512, dtype=BF, device='cuda')
        w = torch.empty(1024, 512, dtype=BF, device='cuda')
        assert torch.ops.ctclip.gemm_bf16(x, w).dtype == BF
        r = torch.empty(256, 1024, dtype=F32, device='cuda')
        y = torch.ops.ctclip.gemm_bf16(x, w, None, r)
        assert y.shape == (256, 1024) and y.dtype == F32
        xf = torch.empty(300, 512, device='cuda')
        g = torch.empty(512, device='cuda')
        yl, m, s = torch.ops.ctclip.layernorm(xf, g, g, 1e-5)
        assert yl.shape == xf.shape and m.shape == s.shape == (300,)
        q = torch.empty(4 * 64, 8 * 32, dtype=BF, device='cuda')
        sc = torch.empty(32, device='cuda')
        o, lse = torch.ops.ctclip.cos_attn(q, q, q, sc, sc, 8, 64, [1, 64, 0, 1], 8.0, None, [0, 0])
        assert o.shape == q.shape and lse.shape == (8, 256)
        t = torch.empty(8, 512, device='cuda')
        lt = torch.empty(1, device='cuda')
        loss, dt, di, dlt = torch.ops.ctclip.clip_infonce(t, t, lt)
        assert loss.shape == () and dt.shape == t.shape and dlt.shape == lt.shape
        idx, xn = torch.ops.ctclip.vq_cos_argmax(xf, torch.empty(8192, 512, device='cuda'))
        assert idx.shape == (300,) and idx.dtype == torch.int32 and xn.shape == xf.shape
        xp = torch.empty(2 * 3 * 4 * 5, 64, device='cuda')
        assert torch.ops.ctclip.peg_dwconv3d(xp, torch.empty(64, 1, 3, 3, 3, device='cuda'),
                                             torch.empty(64, device='cuda'), [2, 3, 4, 5], 1).shape == xp.shape
        rel_ = torch.empty(2209, 2, device='cuda')
        u, _, _ = torch.ops.ctclip.cpb_mlp(rel_, torch.empty(512, 2, device='cuda'), g, torch.empty(512, 512, device='cuda'),
                                           g, torch.empty(8, 512, device='cuda'), torch.empty(8, device='cuda'))
        assert u.shape == (8, 2209)
        vol = torch.empty(2, 1, 20, 80, 80, dtype=torch.int16, device='cuda')
        pw = torch.empty(512, 4000, device='cuda')
        p1 = torch.empty(4000, device='cuda')
        ye = torch.ops.ctclip.patch_embed_i16(vol, p1, p1, pw, g, g, g, 10, 20)
        assert ye[0].shape == (64, 512) and ye[1].shape == (64, 4032) and ye[1].dtype == BF
        xb_ = torch.empty(2, 16, 256, device='cuda')
        wl = [torch.empty(256, 256, device='cuda'), torch.empty(256, device='cuda')]
        bl = torch.ops.ctclip.bert_layer(xb_, torch.empty(2, 16, dtype=torch.int64, device='cuda'), 4, 1e-12,
                                         *(wl * 4), wl[1], wl[1], torch.empty(1024, 256, device='cuda'),
                                         torch.empty(1024, device='cuda'), torch.empty(256, 1024, device='cuda'),
                                         wl[1], wl[1], wl[1])
        assert bl.shape == xb_.shape


def test_ops_refuse_host_tensors():
    """Registered for the HIP ("cuda") device type only: no silent CPU path."""
    with pytest.raises(NotImplementedError):
        torch.ops.ctclip.gemm_bf16(torch.zeros(4, 4, dtype=BF), torch.zeros(4, 4, dtype=BF))
    with pytest.raises(NotImplementedError):
        ops.layernorm(torch.zeros(2, 8), torch.ones(8), torch.zeros(8))


# ------------------------------------------------------------------------------ GPU numerics
dev = 'cuda'


@pytest.mark.gpu
@pytest.mark.parametrize('bias,res', [(False, False), (True, True)])
def test_gemm_bf16_fwd_bwd(bias, res):
    g = torch.Generator(device=dev).manual_seed(1)
    M, Kd, N = 1024, 512, 768
    x = torch.randn(M, Kd, device=dev, generator=g).to(BF).requires_grad_(True)
    w = (torch.randn(N, Kd, device=dev, generator=g) / Kd ** 0.5).to(BF).requires_grad_(True)
    b = torch.randn(N, device=dev, generator=g).requires_grad_(True) if bias else None
    r = torch.randn(M, N, device=dev, generator=g).requires_grad_(True) if res else None
    y = ops.gemm_bf16(x, w, b, r)
    assert y.dtype == (F32 if res else BF)
    xr, wr = x.detach().float().requires_grad_(True), w.detach().float().requires_grad_(True)
    br = b.detach().clone().requires_grad_(True) if bias else None
    rr = r.detach().clone().requires_grad_(True) if res else None
    yr = F.linear(xr, wr, br) + (rr if res else 0)
    assert rel(y.float(), yr) < 1e-2
    dy = torch.randn(M, N, device=dev, generator=g).to(y.dtype)
    y.backward(dy)
    yr.backward(dy.float())
    assert rel(x.grad.float(), xr.grad) < 1e-2 and x.grad.dtype == BF
    assert rel(w.grad.float(), wr.grad) < 1e-2 and w.grad.dtype == BF
    if bias:
        assert rel(b.grad, br.grad) < 1e-5
    if res:
        assert torch.equal(r.grad, dy)


@pytest.mark.gpu
def test_layernorm_fwd_bwd():
    g = torch.Generator(device=dev).manual_seed(2)
    x = (torch.randn(3000, 512, device=dev, generator=g) * 3 + 1).requires_grad_(True)
    gam = (1 + 0.1 * torch.randn(512, device=dev, generator=g)).requires_grad_(True)
    bet = (0.1 * torch.randn(512, device=dev, generator=g)).requires_grad_(True)
    y = ops.layernorm(x, gam, bet, 1e-5)
    xr, gr, br = (t.detach().clone().requires_grad_(True) for t in (x, gam, bet))
    yr = F.layer_norm(xr, (512,), gr, br, 1e-5)
    assert rel(y, yr) < 1e-5
    dy = torch.randn_like(y)
    y.backward(dy)
    yr.backward(dy)
    for a, b in ((x, xr), (gam, gr), (bet, br)):
        assert rel(a.grad, b.grad) < 1e-4


def _attn_ref(q, k, v, qs, ks, H, L, scale, bias, grid, layout):
    M, HD = q.shape
    D = HD // H
    n_in, s_out, s_in, s_pos = layout
    s = torch.arange(M // L, device=q.device)
    rows = ((s // n_in) * s_out + (s % n_in) * s_in)[:, None] + torch.arange(L, device=q.device)[None] * s_pos

    def heads(t):
        return t.float()[rows].view(M // L, L, H, D).transpose(1, 2)
    qn = F.normalize(heads(q), dim=-1) * qs
    kn = F.normalize(heads(k), dim=-1) * ks
    sim = qn @ kn.transpose(-1, -2) * scale
    if bias is not None:
        gh, gw = grid
        p = torch.arange(L, device=q.device)
        dh = (p // gw)[:, None] - (p // gw)[None]
        dw = (p % gw)[:, None] - (p % gw)[None]
        sim = sim + bias[:, (dh + gh - 1) * (2 * gw - 1) + dw + gw - 1][None]
    o = sim.softmax(-1) @ heads(v)
    out = torch.empty(M, HD, device=q.device, dtype=o.dtype)
    out[rows.reshape(-1)] = o.transpose(1, 2).reshape(-1, HD)
    return out


@pytest.mark.gpu
@pytest.mark.parametrize('case', ['bert_like', 'spatial_bias', 'temporal'])
def test_cos_attn_fwd_bwd(case):
    g = torch.Generator(device=dev).manual_seed(3)
    H, D = 8, 32
    if case == 'bert_like':
        L, nseq, layout, bias, grid, D = 128, 4, None, None, (0, 0), 64
    elif case == 'spatial_bias':
        L, nseq, layout, grid = 64, 6, None, (8, 8)
        bias = torch.randn(H, 15 * 15, device=dev, generator=g).requires_grad_(True)
    else:   # temporal rows (b, t, h*w): sequences over t, '(b h w) t d' (functional.Geo.seq)
        B, T, HW = 2, 8, 16
        L, nseq, layout, bias, grid = T, B * HW, (HW, T * HW, 1, HW), None, (0, 0)
    M = L * nseq
    q, k, v = ((torch.randn(M, H * D, device=dev, generator=g)).to(BF).requires_grad_(True) for _ in range(3))
    qs = (1 + 0.1 * torch.randn(D, device=dev, generator=g)).requires_grad_(True)
    ks = (1 + 0.1 * torch.randn(D, device=dev, generator=g)).requires_grad_(True)
    scale = 8.0 if case != 'bert_like' else 1 / math.sqrt(D)
    o = ops.cos_attn(q, k, v, qs, ks, H, L, layout, scale, bias, grid)
    lay = layout or (1, L, 0, 1)
    ins = [t.detach().clone().requires_grad_(True) for t in (q, k, v, qs, ks)]
    br = bias.detach().clone().requires_grad_(True) if bias is not None else None
    ref = _attn_ref(*ins, H, L, scale, br, grid, lay)
    assert rel(o.float(), ref) < 1e-2
    do = torch.randn(M, H * D, device=dev, generator=g).to(BF)
    o.backward(do)
    ref.backward(do.float())
    for name, a, b in zip(('q', 'k', 'v', 'q_scale', 'k_scale'), (q, k, v, qs, ks), ins):
        assert rel(a.grad.float(), b.grad) < 3e-2, name
    if bias is not None:
        assert rel(bias.grad, br.grad) < 3e-2


@pytest.mark.gpu
@pytest.mark.parametrize('Bg', [2, 8, 64])
def test_clip_infonce(Bg):
    g = torch.Generator(device=dev).manual_seed(4)
    t = torch.randn(Bg, 512, device=dev, generator=g).requires_grad_(True)
    i = torch.randn(Bg, 512, device=dev, generator=g).requires_grad_(True)
    lt = torch.tensor([math.log(1 / 0.07)], device=dev).requires_grad_(True)
    loss = ops.clip_infonce(t, i, lt)
    tr, ir, lr = (x.detach().clone().requires_grad_(True) for x in (t, i, lt))
    sim = F.normalize(tr, dim=-1) @ F.normalize(ir, dim=-1).t() * lr.exp()
    lab = torch.arange(Bg, device=dev)
    ref = (F.cross_entropy(sim, lab) + F.cross_entropy(sim.t(), lab)) / 2
    assert abs(loss.item() - ref.item()) < 1e-5 * max(1.0, abs(ref.item()))
    (2.0 * loss).backward()
    (2.0 * ref).backward()
    assert rel(t.grad, tr.grad) < 1e-4 and rel(i.grad, ir.grad) < 1e-4 and rel(lt.grad, lr.grad) < 1e-4


@pytest.mark.gpu
def test_vq_cos_argmax():
    g = torch.Generator(device=dev).manual_seed(5)
    x = torch.randn(4000, 512, device=dev, generator=g)
    cb = F.normalize(torch.randn(8192, 512, device=dev, generator=g), dim=-1)
    idx, xn = ops.vq_cos_argmax(x, cb)
    s64 = F.normalize(x.double(), dim=-1) @ cb.double().t()
    top2 = s64.topk(2, dim=1).values
    tie = (top2[:, 0] - top2[:, 1]) < 1e-6          # only f32-level ties may differ
    assert (idx.long() != s64.argmax(1))[~tie].sum().item() == 0
    assert rel(xn, F.normalize(x, dim=-1)) < 1e-6


def _peg_torch(x, w, b, shape, mode):
    """x + causal depthwise conv3d in the reference's view (attention.py:56-84; mode 1 views the
    '(b h w) t d' tensor through a raw reshape to (b, t, h, w))."""
    B, T, H, W = shape
    D = x.shape[1]
    if mode == 1:
        xv = x.reshape(B, T, H, W, D).permute(0, 2, 3, 1, 4).reshape(B, T, H, W, D)   # raw reshape
    else:
        xv = x.reshape(B, T, H, W, D)
    v = F.pad(xv.permute(0, 4, 1, 2, 3), (1, 1, 1, 1, 2, 0))
    y = F.conv3d(v, w, b, groups=D).permute(0, 2, 3, 4, 1)
    if mode == 1:
        y = y.reshape(B, H, W, T, D).permute(0, 3, 1, 2, 4)
    return x + y.reshape(-1, D)


@pytest.mark.gpu
@pytest.mark.parametrize('mode', [0, 1])
@pytest.mark.parametrize('shape,D', [((2, 6, 5, 7), 128), ((1, 4, 24, 24), 512)])
def test_peg_dwconv3d(mode, shape, D):
    g = torch.Generator(device=dev).manual_seed(7)
    M = shape[0] * shape[1] * shape[2] * shape[3]
    x = torch.randn(M, D, device=dev, generator=g).bfloat16().float().requires_grad_(True)
    w = (torch.randn(D, 1, 3, 3, 3, device=dev, generator=g) * 0.2).requires_grad_(True)
    b = (torch.randn(D, device=dev, generator=g) * 0.1).requires_grad_(True)
    y = ops.peg_dwconv3d(x, w, b, list(shape), mode)
    xr, wr, br = (t.detach().clone().requires_grad_(True) for t in (x, w, b))
    yr = _peg_torch(xr, wr, br, shape, mode)
    assert rel(y, yr) < 1e-5
    dy = torch.randn(M, D, device=dev, generator=g).bfloat16().float()
    y.backward(dy)
    yr.backward(dy)
    assert rel(x.grad, xr.grad) < 1e-5 and rel(w.grad, wr.grad) < 1e-5 and rel(b.grad, br.grad) < 1e-5


@pytest.mark.gpu
def test_cpb_mlp_and_biased_attention():
    """CPB table from the op feeds cos_attn's bias; gradients flow through both ops back to the
    MLP weights (ContinuousPositionBias -> Attention, attention.py:229-276,160-165)."""
    from ctclip_mi355x import functional as Fn
    g = torch.Generator(device=dev).manual_seed(8)
    gh, gw, H, D, d = 6, 6, 8, 32, 64
    rel_ = Fn.cpb_table(gh, gw, dev)
    ws = [torch.randn(d, 2, device=dev, generator=g) * 0.5, torch.randn(d, device=dev, generator=g) * 0.1,
          torch.randn(d, d, device=dev, generator=g) / 8, torch.randn(d, device=dev, generator=g) * 0.1,
          torch.randn(H, d, device=dev, generator=g) / 8, torch.randn(H, device=dev, generator=g) * 0.1]
    ws = [t.requires_grad_(True) for t in ws]
    u = ops.cpb_mlp(rel_, *ws)
    wr = [t.detach().clone().requires_grad_(True) for t in ws]
    h = F.leaky_relu(F.linear(rel_, wr[0], wr[1]), 0.1)
    h = F.leaky_relu(F.linear(h, wr[2], wr[3]), 0.1)
    ur = F.linear(h, wr[4], wr[5]).t()
    assert rel(u, ur) < 1e-5
    L, nseq = gh * gw, 4
    q, k, v = (torch.randn(L * nseq, H * D, device=dev, generator=g).to(BF) for _ in range(3))
    one = torch.ones(D, device=dev)
    o = ops.cos_attn(q, k, v, one, one, H, L, None, 8.0, u, (gh, gw))
    orf = _attn_ref(q, k, v, one, one, H, L, 8.0, ur, (gh, gw), (1, L, 0, 1))
    assert rel(o.float(), orf) < 1e-2
    do = torch.randn_like(orf)
    o.backward(do.to(BF))
    orf.backward(do.to(BF).float())
    errs = [rel(a.grad, b_.grad) for a, b_ in zip(ws[:5], wr[:5])]
    # the last bias adds a per-head constant to every score, which the softmax cancels: its exact
    # gradient is 0 (the torch reference gives 9e-6), so it is held to the scale of the other grads
    errs.append(((ws[5].grad - wr[5].grad).norm() / wr[4].grad.norm()).item())
    assert max(errs) < 3e-2, errs


@pytest.mark.gpu
def test_opcheck_registrations():
    """torch.library.opcheck: schema, fake tensor and autograd-registration checks on device inputs."""
    g = torch.Generator(device=dev).manual_seed(6)
    x = torch.randn(256, 512, device=dev, generator=g).to(BF)
    w = torch.randn(512, 512, device=dev, generator=g).to(BF)
    utils = ('test_schema', 'test_faketensor', 'test_autograd_registration')
    torch.library.opcheck(torch.ops.ctclip.gemm_bf16, (x, w, None, None), test_utils=utils)
    xf = torch.randn(256, 512, device=dev, generator=g)
    gam = torch.ones(512, device=dev)
    torch.library.opcheck(torch.ops.ctclip.layernorm, (xf, gam, gam * 0, 1e-5), test_utils=utils)
    t = torch.randn(8, 512, device=dev, generator=g)
    torch.library.opcheck(torch.ops.ctclip.clip_infonce, (t, t.flip(0), torch.ones(1, device=dev)),
                          test_utils=utils)


@pytest.mark.gpu
def test_patch_embed_i16_fwd_bwd():
    """to_patch_emb on a raw int16 HU volume (ct_clip/data.py:150-152 + ctvit.py:169-174) against the
    fp32 torch restatement; weight gradients through the op's registered backward."""
    g = torch.Generator(device=dev).manual_seed(9)
    B, Fr, S, PT, P, dim = 2, 20, 80, 10, 20, 512
    pd = PT * P * P
    hu = torch.randint(-1200, 1200, (B, 1, Fr, S, S), device=dev, dtype=torch.int16, generator=g)
    ws = [torch.randn(pd, device=dev, generator=g) * 0.1 + 1, torch.randn(pd, device=dev, generator=g) * 0.1,
          torch.randn(dim, pd, device=dev, generator=g) / pd ** 0.5, torch.randn(dim, device=dev, generator=g) * 0.1,
          torch.randn(dim, device=dev, generator=g) * 0.1 + 1, torch.randn(dim, device=dev, generator=g) * 0.1]
    ws = [t.requires_grad_(True) for t in ws]
    y = ops.patch_embed_i16(hu, *ws, PT, P)
    wr = [t.detach().clone().requires_grad_(True) for t in ws]
    v = hu.float().clamp(-1000, 1000) / 1000
    T, Hg, Wg = Fr // PT, S // P, S // P
    p = v.reshape(B, 1, T, PT, Hg, P, Wg, P).permute(0, 2, 4, 6, 1, 3, 5, 7).reshape(-1, pd)
    yr = F.layer_norm(F.linear(F.layer_norm(p, (pd,), wr[0], wr[1], 1e-5), wr[2], wr[3]), (dim,), wr[4], wr[5], 1e-5)
    assert y.shape == (B * T * Hg * Wg, dim)
    assert rel(y, yr) < 1e-2, rel(y, yr)
    dy = torch.randn_like(yr)
    y.backward(dy)
    yr.backward(dy)
    errs = [rel(a.grad, b_.grad) for a, b_ in zip(ws, wr)]
    assert max(errs) < 3e-2, errs


def _bert_layer_ref(x, mask, heads, eps, wq, bq, wk, bk, wv, bv, wo, bo, g1, b1, wi, bi, wout, bout, g2, b2):
    """HF BertLayer (eval, post-LN, exact GELU) in fp32 torch."""
    B, L, Hd = x.shape
    dh = Hd // heads
    sp = lambda t: t.view(B, L, heads, dh).transpose(1, 2)  # noqa: E731
    q, k, v = sp(F.linear(x, wq, bq)), sp(F.linear(x, wk, bk)), sp(F.linear(x, wv, bv))
    s = q @ k.transpose(-1, -2) / math.sqrt(dh) + (1 - mask.float())[:, None, None, :] * -1e30
    c = (s.softmax(-1) @ v).transpose(1, 2).reshape(B, L, Hd)
    a = F.layer_norm(F.linear(c, wo, bo) + x, (Hd,), g1, b1, eps)
    return F.layer_norm(F.linear(F.gelu(F.linear(a, wi, bi)), wout, bout) + a, (Hd,), g2, b2, eps)


@pytest.mark.gpu
@pytest.mark.parametrize('Hd,heads,inter', [(768, 12, 3072), (256, 8, 1024)])
def test_bert_layer(Hd, heads, inter):
    """One BertLayer forward (the text tower's unit, ct_clip/ct_clip.py:685-686) with a padded key mask
    against the fp32 restatement: the hi / lo split-weight GEMMs keep it at the 1e-3 level."""
    g = torch.Generator(device=dev).manual_seed(10)
    B, L = 4, 128
    r = lambda *s, sc=0.02: torch.randn(*s, device=dev, generator=g) * sc  # noqa: E731
    ws = [r(Hd, Hd), r(Hd), r(Hd, Hd), r(Hd), r(Hd, Hd), r(Hd), r(Hd, Hd), r(Hd), 1 + r(Hd, sc=0.1), r(Hd),
          r(inter, Hd), r(inter), r(Hd, inter), r(Hd), 1 + r(Hd, sc=0.1), r(Hd)]
    x = torch.randn(B, L, Hd, device=dev, generator=g)
    mask = torch.ones(B, L, device=dev, dtype=torch.int64)
    mask[1, 90:] = 0
    mask[3, 17:] = 0
    y = torch.ops.ctclip.bert_layer(x, mask, heads, 1e-12, *ws)
    yr = _bert_layer_ref(x, mask, heads, 1e-12, *ws)
    assert y.shape == x.shape
    assert rel(y, yr) < 3e-3, rel(y, yr)
