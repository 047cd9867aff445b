"""The 3D-ViT forward's fp16 GEMMs (round 5, functional.vit_f16): fp16 A / B operands
of the patch embedding, the LayerNorm-folded Q | K | V projection, to_out (+ the FeedForward
LayerNorm) and FF1 (ct_clip/ctvit.py:169-174, ct_clip/attention.py:44-52,119-125,139-143), their
producers' fp16 copies (patch LayerNorm, PEG, attention output, LayerNorm), the fp16 h of the GEGLU
epilogue and its backward reader -- each against an f64 evaluation on the same fp16 operands -- and a
whole layer pair: the fp16 forward is closer to the fp32 torch reference than the bf16 one."""
import pytest
import torch
import torch.nn.functional as F

from oracle import ctclip_oracle as O

pytestmark = pytest.mark.gpu
F16 = torch.float16


@pytest.fixture(scope='module')
def K():
    from ctclip_mi355x import kernels
    return kernels


def _rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize('M,N,Kd', [(110592, 512, 4032), (4096, 768, 512), (300, 512, 256)])
def test_f16_linear_epilogues(K, M, N, Kd):
    """Plain 16-bit output, f32 + bias (the patch embedding), f32 residual + bf16 shadow (to_out
    unfused): 8-phase kernel at large M, 128-tile kernel at M = 300."""
    g = torch.Generator(device='cuda').manual_seed(1)
    x = torch.randn(M, Kd, device='cuda', generator=g).half()
    w = (torch.randn(N, Kd, device='cuda', generator=g) / Kd ** 0.5).half()
    b = torch.randn(N, device='cuda', generator=g) * 0.1
    r = torch.randn(M, N, device='cuda', generator=g)
    ref = x.double() @ w.double().t()
    y = K.linear(x, w)
    assert y.dtype == torch.bfloat16 and _rel(y, ref) < 4e-3
    yb = K.linear(x, w, bias=b, out_dtype=torch.float32)
    assert _rel(yb, ref + b.double()) < 1e-5
    sh = torch.empty(M, N, device='cuda', dtype=torch.bfloat16)
    yr = K.linear(x, w, residual=r, out_dtype=torch.float32, out2=sh)
    assert _rel(yr, ref + r.double()) < 1e-5
    assert torch.equal(sh, yr.bfloat16())
    # the fp16 operands are what buys the accuracy: same data through bf16 operands is ~8x worse
    xf, wf = torch.randn(M, Kd, device='cuda', generator=g), torch.randn(N, Kd, device='cuda', generator=g)
    e16 = _rel(K.linear(xf.half(), wf.half(), out_dtype=torch.float32), xf.double() @ wf.double().t())
    e16b = _rel(K.linear(xf.bfloat16(), wf.bfloat16(), out_dtype=torch.float32), xf.double() @ wf.double().t())
    print(f'M={M} N={N} K={Kd}: fp16-operand GEMM rel err {e16:.2e}, bf16 {e16b:.2e}')
    assert e16 < e16b / 4


@pytest.mark.parametrize('M', [8192, 300])
def test_f16_geglu_h_and_backward(K, M):
    """act 2 on fp16 operands: h stored in fp16 in the derivative form [gelu(gate) | x gelu'(gate)]
    (round 6), g = gelu(gate) x from the fp16-rounded x / gate (bf16); act 4 reads that fp16 h (r_f16) and
    multiplies dg by its two factors -- against the stored factors and against the f64 truth (the
    GEGLU derivative at the exact pre-activation).  M = 300 takes the 128-tile kernel."""
    g_ = torch.Generator(device='cuda').manual_seed(2)
    N, Kd = 2816, 512
    x = torch.randn(M, Kd, device='cuda', generator=g_).half()
    w = (torch.randn(N, Kd, device='cuda', generator=g_) * 0.05).half()
    gout = torch.empty(M, N // 2, device='cuda', dtype=torch.bfloat16)
    h = K.linear(x, w, act=K.ACT_GEGLU, out2=gout, out_dtype=F16)
    assert h.dtype == F16
    hp = (x.double() @ w.double().t()).view(M, N // 64, 2, 32)
    xp, gp = hp[:, :, 0], hp[:, :, 1]
    cdf = 0.5 * (1 + torch.erf(gp / 2 ** 0.5))
    pdf = torch.exp(-0.5 * gp * gp) / (2 * torch.pi) ** 0.5
    hd = torch.stack([F.gelu(gp), xp * (cdf + gp * pdf)], 2).reshape(M, N)
    assert _rel(h, hd) < 1e-3
    gref = (F.gelu(gp) * xp).reshape(M, N // 2)
    assert _rel(gout, gref) < 4e-3
    # the GEGLU backward on the fp16 h
    D, G = 512, N // 2
    dy = (torch.randn(M, D, device='cuda', generator=g_) * 0.1).bfloat16()
    w2p = (torch.randn(D, G, device='cuda', generator=g_) * 0.05).bfloat16()
    dh = K.matmul_nn_geglu_bwd(dy, w2p, h)
    dg = (dy.float() @ w2p.float()).bfloat16().float()
    d = dg.view(M, G // 32, 32)
    hv = h.float().view(M, N // 64, 2, 32)
    refm = torch.stack([d * hv[:, :, 0], d * hv[:, :, 1]], 2).reshape(M, 2 * G)
    assert _rel(dh, refm) < 8e-3                     # the products, bf16-rounded
    truth = torch.stack([d * F.gelu(gp), d * xp * (cdf + gp * pdf)], 2).reshape(M, 2 * G)
    assert _rel(dh, truth) < 1e-2


def test_f16_residual_ln_y16(K):
    """ctclip_gemm_ln mode 1 on fp16 operands with the fp16 copy of the LayerNorm output."""
    g = torch.Generator(device='cuda').manual_seed(3)
    M, Kd = 16384, 256
    o = torch.randn(M, Kd, device='cuda', generator=g).half()
    W = (torch.randn(512, Kd, device='cuda', generator=g) / Kd ** 0.5).half()
    res = torch.randn(M, 512, device='cuda', generator=g) + 0.3
    gamma = 1 + 0.1 * torch.randn(512, device='cuda', generator=g)
    beta = 0.1 * torch.randn(512, device='cuda', generator=g)
    with K.ln_guard():
        out = K.linear_residual_ln(o, W, res, gamma, beta, 1e-5, y16=True)
    assert out is not None
    x1f, x1b, y, mean, rstd, yh = out
    assert _rel(x1f, o.double() @ W.double().t() + res.double()) < 1e-5
    ln = F.layer_norm(x1f, (512,), gamma, beta, 1e-5)
    assert _rel(yh, ln) < 1e-3 and _rel(y, ln) < 4e-3
    assert (yh.float() - ln).abs().max().item() <= 2 ** -10 * ln.abs().max().item() * 1.01
    assert K.ln_fused_status() == 0


@pytest.mark.parametrize('M,shift', [(4096, 0.4), (110592, 0.4), (4096, 30.0)])
def test_f16_qkv_lnfold(K, M, shift):
    """The LayerNorm-folded Q | K | V GEMM on fp16 operands.  shift = 30: a residual stream with a
    per-row mean 30x its spread (a trained-model statistic): the fold computes
    rstd (x (g o Wq)^T - mean cs) from the fp16 x, so its Q error grows with |mean| / std -- printed
    beside the plain case, bound stated below."""
    g = torch.Generator(device='cuda').manual_seed(4)
    x1f = torch.randn(M, 512, device='cuda', generator=g) * 1.3 + shift
    Wq = torch.randn(256, 512, device='cuda', generator=g) / 512 ** 0.5
    Wkv = torch.randn(512, 512, device='cuda', generator=g) / 512 ** 0.5
    gamma = 1 + 0.2 * torch.randn(512, device='cuda', generator=g)
    qs = 1 + 0.1 * torch.randn(32, device='cuda', generator=g)
    ks = 1 + 0.1 * torch.randn(32, device='cuda', generator=g)
    _, _, mean, rstd = K.layernorm_fwd(x1f, gamma, None, 1e-5)
    _, _, scales = K.pack_qkv_fold(Wq, gamma, Wkv.bfloat16(), qs, ks)
    Wp, cs = K.pack_qkv_fold_h16(Wq, gamma, Wkv)
    wf = (Wq * gamma).half()
    assert torch.equal(Wp[:256], wf) and torch.equal(Wp[256:], Wkv.half())
    assert _rel(cs, wf.double().sum(1)) < 1e-6
    x1h = x1f.half()
    qkv, qkn = K.linear_qkv_lnfold(x1h, Wp, cs, mean, rstd, scales, 256, 512)
    q_ref = rstd.double()[:, None] * (x1h.double() @ wf.double().t() - mean.double()[:, None] * cs.double()[None])
    assert _rel(qkv[:, :256], q_ref) < 3e-3
    assert _rel(qkv[:, 256:], x1h.double() @ Wkv.half().double().t()) < 3e-3
    # torch fp32 semantics: l2norm(LayerNorm(x) Wq^T) * q_scale, closer than the bf16 fold allows
    q32 = F.layer_norm(x1f.double(), (512,), gamma.double(), None, 1e-5) @ Wq.double().t()
    h = q32.view(M, 8, 32)
    qn32 = (h / h.norm(dim=-1, keepdim=True) * qs.double()).view(M, 256)
    eq = _rel(qkn[:, :256], qn32)
    # the unfolded fp16 path for comparison: LayerNorm in f32, then its fp16 output times fp16 Wq, the
    # l2norm stored in bf16 as the fold's C2 is (the bf16 storage alone is ~2e-3 of this error)
    ln16 = F.layer_norm(x1f, (512,), gamma, None, 1e-5).half()
    hu = (ln16.double() @ Wq.half().double().t()).view(M, 8, 32)
    qnu = (hu / hu.norm(dim=-1, keepdim=True) * qs.double()).view(M, 256)
    eu, eub = _rel(qnu, qn32), _rel(qnu.bfloat16(), qn32)
    print(f'fold fp16, row mean {shift}: l2norm(q) rel err vs f64 {eq:.2e} (unfolded fp16 LayerNorm {eu:.2e}, '
          f'{eub:.2e} with the same bf16 output)')
    assert eq < (5e-3 if shift < 1 else 2e-2)


def test_f16_producer_copies(K):
    """The fp16 copies written beside the bf16 outputs: LayerNorm forward (== its f32 output rounded),
    patch LayerNorm (zero K padding), attention output."""
    g = torch.Generator(device='cuda').manual_seed(5)
    x = torch.randn(5000, 512, device='cuda', generator=g) * 2 + 1
    gm = 1 + 0.1 * torch.randn(512, device='cuda', generator=g)
    bt = 0.1 * torch.randn(512, device='cuda', generator=g)
    yb, yf, _, _, yh = K.layernorm_fwd(x, gm, bt, 1e-5, out_f32=True, out_f16=True)
    assert torch.equal(yh, yf.half()) and torch.equal(yb, yf.bfloat16())
    from ctclip_mi355x.layers import patch_offsets
    hu = torch.randint(-1200, 1201, (1, 1, 40, 160, 160), dtype=torch.int16, device='cuda', generator=g)
    offs = patch_offsets(1, 10, 20, 40, 160, 160).cuda()
    xb, xh = K.patch_ln(hu, True, 10, 20, offs, ld=4032, want_f16=True)
    assert torch.equal(xb, K.patch_ln(hu, True, 10, 20, offs, ld=4032))
    assert (xh[:, 4000:] == 0).all()
    assert ((xh.float() - xb.float()).abs() <= 2 ** -8 * xb.float().abs() + 1e-6).all()
    M, H, D = 3 * 576, 8, 32
    q = F.normalize(torch.randn(M, H, D, device='cuda', generator=g), dim=-1).view(M, H * D).bfloat16()
    kv = torch.randn(M, 2 * H * D, device='cuda', generator=g).bfloat16()
    o, _, o16 = K.attn_fwd(q, kv[:, :256], kv[:, 256:], L=576, H=H, D=D, nseq=3, scale=8.0, seq=(1, 576, 0, 1),
                           want_o16=True)
    o_only, _ = K.attn_fwd(q, kv[:, :256], kv[:, 256:], L=576, H=H, D=D, nseq=3, scale=8.0, seq=(1, 576, 0, 1))
    assert torch.equal(o, o_only)
    assert ((o16.float() - o.float()).abs() <= 2 ** -8 * o.float().abs() + 1e-6).all()


@pytest.mark.parametrize('mode', [0, 1])
def test_f16_layers_closer_to_fp32(K, mode):
    """Two 3D-ViT layers + norm_out at B = 1 on the 24^3 grid: the fp16 forward's output is much closer
    to the fp32 torch reference (oracle.transformer_forward) than the bf16 forward's, and its
    gradients stay within the bf16 backward's tolerance of each other."""
    from ctclip_mi355x import attention as A, functional as Fn
    torch.manual_seed(6)
    tr = A.Transformer(512, depth=2, dim_head=32, heads=8).cuda()
    with torch.no_grad():
        for p in tr.parameters():
            p.add_(0.02 * torch.randn_like(p))
    geo = Fn.Geo(B=1, T=24, Hg=24, Wg=24, heads=8, dim_head=32, mode=mode)
    xf0 = torch.randn(geo.M, 512, device='cuda')
    sd = {k: v.detach() for k, v in tr.state_dict().items()}
    shape = (1, 24, 24, 24)
    if mode == 0:
        ref = O.transformer_forward(sd, '', xf0.view(24, 576, 512), 2, 8, 32, shape).reshape(-1, 512)
    else:
        xt = xf0.view(1, 24, 24, 24, 512).permute(0, 2, 3, 1, 4).reshape(576, 24, 512)
        ref = O.transformer_forward(sd, '', xt, 2, 8, 32, shape)
        ref = ref.reshape(1, 24, 24, 24, 512).permute(0, 3, 1, 2, 4).reshape(-1, 512)
    dy = torch.randn(geo.M, 512, device='cuda') * 1e-2
    outs = {}
    prev = Fn.set_vit_f16(True)
    try:
        for on in (True, False):
            Fn.set_vit_f16(on)
            for p in tr.parameters():
                p.grad = None
            xf = xf0.clone().requires_grad_(True)
            yf, _ = tr.run(xf, xf0.bfloat16(), geo)
            yf.backward(dy)
            torch.cuda.synchronize()
            outs[on] = (yf.detach(), xf.grad, {n: p.grad.clone() for n, p in tr.named_parameters()
                                               if p.grad is not None})
    finally:
        Fn.set_vit_f16(prev)
    e16, e_bf = _rel(outs[True][0], ref), _rel(outs[False][0], ref)
    print(f'mode {mode}: layer output rel err vs fp32: fp16 forward {e16:.2e}, bf16 forward {e_bf:.2e}')
    assert e16 < 0.7 * e_bf
    assert _rel(outs[True][1], outs[False][1]) < 3e-2
    for n, gr in outs[False][2].items():
        assert _rel(outs[True][2][n], gr) < 5e-2, n


@pytest.mark.parametrize('M,G', [(8192, 1408), (8000, 1376), (4100, 1408)])
def test_geglu_bwd_epilogue_bounds(K, M, G):
    """The r05ab fault: a diagnostic build that prefetched the GEGLU-backward
    epilogue's h lines faulted on test_f16_geglu_h_and_backward[8192].  The shipped epilogue reads h
    only for rows < M and g-space column groups t with 32 t < N (the waves of the last 256-column tile
    past N = 1,408 read and write nothing).  Here h and dh are views into wider buffers: the padding of
    h holds NaN (a read past column 2G would reach dh) and the padding of dh a sentinel (a write past
    it would change it); M and G not multiples of the 256-tile, both fp16 and bf16 h."""
    g_ = torch.Generator(device='cuda').manual_seed(21)
    D = 512
    for hdt in (F16, torch.bfloat16):
        hbuf = torch.full((M, 2 * G + 64), float('nan'), device='cuda', dtype=hdt)
        h = hbuf[:, :2 * G]
        h.copy_(torch.randn(M, 2 * G, device='cuda', generator=g_).to(hdt))
        dbuf = torch.full((M, 2 * G + 64), 7.0, device='cuda', dtype=torch.bfloat16)
        dh = dbuf[:, :2 * G]
        dy = (torch.randn(M, D, device='cuda', generator=g_) * 0.1).bfloat16()
        w2p = (torch.randn(D, G, device='cuda', generator=g_) * 0.05).bfloat16()
        K.matmul_nn_geglu_bwd(dy, w2p, h, out=dh)
        torch.cuda.synchronize()
        assert (dbuf[:, 2 * G:] == 7.0).all()
        assert torch.isfinite(dh.float()).all()
        hv = h.float().view(M, G // 32, 2, 32)
        xg, gt = hv[:, :, 0], hv[:, :, 1]
        d = (dy.float() @ w2p.float()).bfloat16().float().view(M, G // 32, 32)
        if hdt == F16:     # fp16 h: the derivative form [gelu(gate) | x gelu'(gate)] (round 6)
            refm = torch.stack([d * xg, d * gt], 2).reshape(M, 2 * G)
        else:
            cdf = 0.5 * (1 + torch.erf(gt / 2 ** 0.5))
            pdf = torch.exp(-0.5 * gt * gt) / (2 * torch.pi) ** 0.5
            refm = torch.stack([d * F.gelu(gt), d * xg * (cdf + gt * pdf)], 2).reshape(M, 2 * G)
        assert _rel(dh, refm) < 1e-2
