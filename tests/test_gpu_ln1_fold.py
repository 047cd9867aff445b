"""The attention's pre-norm LayerNorm folded into one Q | K | V projection (gemm256.hip EP 8,
ctclip_gemm_qkv_lnfold; ct_clip/attention.py:139-141 norm -> to_q, 119-125 to_q / to_kv, 152-154
l2norm * scale): the PEG forward's row statistics (ctclip_peg_fwd_stats + ctclip_ln_stats_merge),
the packed B operand, the fused projection against an f64 evaluation of the fold on the same bf16
operands and against the unfused LayerNorm + projections, the Q weight-gradient fold
(ctclip_l2norm_scale_bwd_fold + ctclip_lnfold_wgrad), and whole 3D-ViT layers (spatial and
temporal geometry) with the fold against the unfused kernels."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def K():
    from ctclip_mi355x import kernels
    return kernels


def _rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize('mode', [0, 1])
def test_peg_fwd_stats(K, mode):
    g = torch.Generator(device='cuda').manual_seed(11 + mode)
    B, T, H, W, D = 2, 24, 24, 24, 512
    M = B * T * H * W
    xf = torch.randn(M, D, device='cuda', generator=g) * 1.5 + 0.7          # non-zero row means
    xb = xf.bfloat16()
    w = torch.randn(D, 27, device='cuda', generator=g) * 0.1
    b = torch.randn(D, device='cuda', generator=g) * 0.1
    of0, ob0 = K.peg_fwd(xb, xf, B, T, H, W, w, b, mode)
    of1, ob1, mean, rstd = K.peg_fwd_stats(xb, xf, B, T, H, W, w, b, mode)
    assert torch.equal(of0, of1) and torch.equal(ob0, ob1)
    mu = of0.double().mean(1)
    var = of0.double().var(1, unbiased=False)
    assert ((mean.double() - mu).abs() / var.sqrt()).max().item() < 1e-5
    ref = (var + 1e-5).rsqrt()
    assert ((rstd.double() - ref).abs() / ref).max().item() < 1e-5
    # the LayerNorm kernel's statistics of the same rows
    _, _, m_ln, r_ln = K.layernorm_fwd(of0, torch.ones(D, device='cuda'), None, 1e-5)
    assert ((mean - m_ln).abs() / var.sqrt().float()).max().item() < 1e-5
    assert ((rstd - r_ln).abs() / r_ln).max().item() < 1e-5


def _fold_case(M, seed):
    g = torch.Generator(device='cuda').manual_seed(seed)
    x1f = torch.randn(M, 512, device='cuda', generator=g) * 1.3 + 0.4
    x1b = x1f.bfloat16()
    Wq = torch.randn(256, 512, device='cuda', generator=g) / 512 ** 0.5
    Wkv = (torch.randn(512, 512, device='cuda', generator=g) / 512 ** 0.5).bfloat16()
    gamma = 1 + 0.2 * torch.randn(512, device='cuda', generator=g)
    qs = 1 + 0.1 * torch.randn(32, device='cuda', generator=g)
    ks = 1 + 0.1 * torch.randn(32, device='cuda', generator=g)
    return x1f, x1b, Wq, Wkv, gamma, qs, ks


def _l2n(t, s):
    M, n = t.shape
    h = t.view(M, n // 32, 32)
    return (h / h.norm(dim=-1, keepdim=True).clamp_min(1e-12) * s).view(M, n)


@pytest.mark.parametrize('M', [4096, 110592])
def test_qkv_lnfold_gemm(K, M):
    x1f, x1b, Wq, Wkv, gamma, qs, ks = _fold_case(M, 5)
    _, _, mean, rstd = K.layernorm_fwd(x1f, gamma, None, 1e-5)
    Wp, cs, scales = K.pack_qkv_fold(Wq, gamma, Wkv, qs, ks)
    wf = (Wq * gamma).bfloat16()
    assert torch.equal(Wp[:256], wf) and torch.equal(Wp[256:], Wkv)
    assert _rel(cs, wf.double().sum(1)) < 1e-6
    assert torch.equal(scales, torch.cat([qs, ks]))
    qkv, qkn = K.linear_qkv_lnfold(x1b, Wp, cs, mean, rstd, scales, 256, 512)
    torch.cuda.synchronize()
    # f64 evaluation of the fold on the same bf16 operands
    q_ref = rstd.double()[:, None] * (x1b.double() @ wf.double().t() - mean.double()[:, None] * cs.double()[None])
    assert _rel(qkv[:, :256], q_ref) < 3e-3
    assert _rel(qkn[:, :256], _l2n(qkv[:, :256].double(), qs.double())) < 3e-3
    # K / V columns: the unfused act-5 projection of the same rows -- bit-identical where that also
    # runs on the 8-phase kernel (full size; small M takes the 128-tile kernel, other sum order)
    kn_un = torch.empty(M, 256, device='cuda', dtype=torch.bfloat16)
    kv_un = K.linear(x1b, Wkv, out2=kn_un, l2n_scale=ks, l2n_cols=256)
    if M >= 65536:
        assert torch.equal(qkv[:, 256:], kv_un) and torch.equal(qkn[:, 256:], kn_un)
    assert _rel(qkv[:, 256:], kv_un) < 1e-5 and _rel(qkn[:, 256:], kn_un) < 1e-5
    # against the unfused LayerNorm (f32 rows) -> bf16 -> projection
    xn, _, _, _ = K.layernorm_fwd(x1f, gamma, None, 1e-5)
    qn_un = torch.empty(M, 256, device='cuda', dtype=torch.bfloat16)
    q_un = K.linear(xn, Wq.bfloat16(), out2=qn_un, l2n_scale=qs, l2n_cols=256)
    assert _rel(qkv[:, :256], q_un) < 1e-2
    assert _rel(qkn[:, :256], qn_un) < 1e-2
    # torch fp32 module semantics: l2norm(LayerNorm(x) Wq^T) * q_scale
    q32 = torch.nn.functional.layer_norm(x1f, (512,), gamma, None, 1e-5) @ Wq.t()
    assert _rel(qkn[:, :256], _l2n(q32, qs)) < 1e-2


def test_l2norm_bwd_fold_and_wgrad(K):
    M = 8192
    x1f, x1b, Wq, Wkv, gamma, qs, ks = _fold_case(M, 7)
    _, _, mean, rstd = K.layernorm_fwd(x1f, gamma, None, 1e-5)
    g = torch.Generator(device='cuda').manual_seed(8)
    q = (torch.randn(M, 256, device='cuda', generator=g) * 0.5).bfloat16()
    dqn = (torch.randn(M, 256, device='cuda', generator=g) * 0.1).bfloat16()
    dq0 = torch.empty_like(q)
    ds0 = K.l2norm_scale_bwd(q, dqn, 8, 32, qs, dq0)
    dq1 = torch.empty_like(q)
    Wp, cs, _ = K.pack_qkv_fold(Wq, gamma, Wkv, qs, ks)
    ds1, dq2, u, c1, be = K.l2norm_scale_bwd_fold(q, dqn, 8, 32, qs, rstd, mean, out=dq1, fold_cs=cs, Dm=512)
    torch.cuda.synchronize()
    assert torch.equal(dq0, dq1) and torch.equal(ds0, ds1)
    ref2 = (dq1.float() * rstd[:, None]).bfloat16()
    assert (dq2.float() - ref2.float()).abs().max().item() <= 2 ** -7 * ref2.float().abs().max().item()
    assert _rel(u, (dq2.double() * mean.double()[:, None]).sum(0)) < 1e-5
    al = (dq2.double() @ cs.double()) / 512
    be_ref = rstd.double() * (dq2.double() * q.double()).sum(1) / 512
    assert _rel(be, be_ref) < 1e-5 and _rel(c1, al - be_ref * mean.double()) < 1e-5
    # the folded weight gradients against dq^T LayerNorm(x) / dkv^T x on the same rows
    dkv = (torch.randn(M, 512, device='cuda', generator=g) * 0.1).bfloat16()
    dqkv = torch.cat([dq2, dkv], 1)
    G = K.matmul_tn(dqkv, x1b)
    gq = torch.zeros(256, 512, device='cuda')
    gg = torch.zeros(512, device='cuda')
    gkv = torch.zeros(512, 512, device='cuda')
    K.lnfold_wgrad(G, u, gamma, gq, wq=Wq, grad_gamma=gg, grad_rest=gkv)
    xh = (x1b.double() - mean.double()[:, None]) * rstd.double()[:, None]
    assert _rel(gq, dq1.double().t() @ (xh * gamma.double())) < 1e-2
    assert _rel(gg, ((dq1.double() @ Wq.double()) * xh).sum(0)) < 1e-2
    assert _rel(gkv, dkv.double().t() @ x1b.double()) < 1e-3
    # the folded LayerNorm backward: dqkv [gamma o Wq ; Wkv] + res - c1 - beta x = LN'(dq Wq) + dkv Wkv + res
    res = torch.randn(M, 512, device='cuda', generator=g)
    dxf, dxb = K.matmul_lnfold_bwd(dqkv, Wp, res, x1b, c1, be)
    torch.cuda.synchronize()
    gdy = (dq1.double() @ Wq.double()) * gamma.double()
    lnb = rstd.double()[:, None] * (gdy - gdy.mean(1, keepdim=True) - xh * (gdy * xh).mean(1, keepdim=True))
    ref = lnb + dkv.double() @ Wkv.double() + res.double()
    assert _rel(dxf, ref) < 1e-2
    assert torch.equal(dxb, dxf.bfloat16())


@pytest.mark.parametrize('mode', [0, 1])
def test_layer_fold_vs_unfolded(K, mode):
    """A 3D-ViT layer at B = 2 with the folded LayerNorm against the LayerNorm kernel + two
    projections: outputs, input and parameter gradients agree to bf16 rounding."""
    from ctclip_mi355x import attention as A, functional as Fn
    torch.manual_seed(0)
    tr = A.Transformer(512, depth=1, dim_head=32, heads=8).cuda()
    with torch.no_grad():
        for p in tr.parameters():
            p.add_(0.02 * torch.randn_like(p))
    geo = Fn.Geo(B=2, T=24, Hg=24, Wg=24, heads=8, dim_head=32, mode=mode)
    xf0 = torch.randn(geo.M, 512, device='cuda') + 0.3
    xb0 = xf0.bfloat16()
    dy = torch.randn(geo.M, 512, device='cuda') * 1e-2
    bias = None
    if mode == 0:
        bias = torch.randn(8, 47 * 47, device='cuda') * 0.5

    def run(fold):
        Fn._LN1_FOLD = fold
        for p in tr.parameters():
            p.grad = None
        xf = xf0.clone().requires_grad_(True)
        yf, yb = tr.run(xf, xb0, geo, bias) if bias is not None else tr.run(xf, xb0, geo)
        yf.backward(dy)
        torch.cuda.synchronize()
        return yf.detach(), xf.grad, [(n, p.grad.clone()) for n, p in tr.named_parameters() if p.grad is not None]

    prev = Fn._LN1_FOLD
    try:
        y0, dx0, g0 = run(False)
        y1, dx1, g1 = run(True)
    finally:
        Fn._LN1_FOLD = prev
    assert _rel(y1, y0) < 2e-3
    assert _rel(dx1, dx0) < 1e-2
    assert [n for n, _ in g0] == [n for n, _ in g1]
    for (n, a), (_, b) in zip(g0, g1):
        assert _rel(b, a) < 3e-2, (n, _rel(b, a))


def test_l2norm_qk_bwd_fold_matches_two_passes(K):
    """The merged q | k l2norm backward (one wave per row) against the q fold pass + the k pass."""
    M = 8192
    x1f, x1b, Wq, Wkv, gamma, qs, ks = _fold_case(M, 9)
    _, _, mean, rstd = K.layernorm_fwd(x1f, gamma, None, 1e-5)
    _, cs, _ = K.pack_qkv_fold(Wq, gamma, Wkv, qs, ks)
    g = torch.Generator(device='cuda').manual_seed(10)
    qkv = (torch.randn(M, 768, device='cuda', generator=g) * 0.5).bfloat16()
    dqk = (torch.randn(M, 512, device='cuda', generator=g) * 0.1).bfloat16()
    out1 = torch.zeros(M, 768, device='cuda', dtype=torch.bfloat16)
    dsq1, dsk1, u1, c11, be1 = K.l2norm_qk_bwd_fold(qkv[:, :512], dqk, qs, ks, rstd, mean, out1[:, :512], cs, 512)
    out0 = torch.zeros(M, 768, device='cuda', dtype=torch.bfloat16)
    dsq0, _, u0, c10, be0 = K.l2norm_scale_bwd_fold(qkv[:, :256], dqk[:, :256], 8, 32, qs, rstd, mean,
                                                    dx2=out0[:, :256], fold_cs=cs, Dm=512)
    dsk0 = K.l2norm_scale_bwd(qkv[:, 256:512], dqk[:, 256:], 8, 32, ks, out0[:, 256:512])
    torch.cuda.synchronize()
    assert torch.equal(out1, out0)
    assert torch.equal(c11, c10) and torch.equal(be1, be0)
    assert _rel(u1, u0) < 1e-5 and _rel(dsq1, dsq0) < 1e-5 and _rel(dsk1, dsk0) < 1e-5


def test_layer_heads16_runs_unfolded(K):
    """heads * dim_head = 512 (heads = 16): the fold's merged q | k l2norm backward is built for 256
    q columns only, so the layer must take the unfolded path even with the fold switched on --
    forward + backward run (no assertion inside the backward) and match the unfolded layer exactly."""
    from ctclip_mi355x import attention as A, functional as Fn
    torch.manual_seed(1)
    tr = A.Transformer(512, depth=1, dim_head=32, heads=16).cuda()
    geo = Fn.Geo(B=1, T=8, Hg=8, Wg=8, heads=16, dim_head=32, mode=0)
    xf0 = torch.randn(geo.M, 512, device='cuda') + 0.3
    xb0 = xf0.bfloat16()
    dy = torch.randn(geo.M, 512, device='cuda') * 1e-2

    def run(fold):
        Fn._LN1_FOLD = fold
        for p in tr.parameters():
            p.grad = None
        xf = xf0.clone().requires_grad_(True)
        yf, _ = tr.run(xf, xb0, geo)
        yf.backward(dy)
        torch.cuda.synchronize()
        return yf.detach(), xf.grad

    prev = Fn._LN1_FOLD
    try:
        y0, dx0 = run(False)
        y1, dx1 = run(True)
    finally:
        Fn._LN1_FOLD = prev
    assert torch.isfinite(y1).all() and torch.isfinite(dx1).all()
    assert torch.equal(y1, y0) and torch.equal(dx1, dx0)
