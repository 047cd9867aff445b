"""LayerNorm fused into the N = 512 GEMM epilogues (gemm256.hip EP -6 / -7, ctclip_gemm_ln):
the two 256-column tiles of a row block exchange per-row statistics inside the launch.
Forward (to_out + residual + FeedForward LayerNorm, ct_clip/attention.py:47,324-326) and backward
(dX GEMM + LayerNorm backward + residual) against torch fp32 references of the same op and
against the unfused GEMM + LayerNorm kernel pair; repeated launches are bit-identical and no
launch reports a missing partner (status word)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def K():
    from ctclip_mi355x import kernels
    prev = kernels.LN_FUSED_BWD
    kernels.LN_FUSED_BWD = True      # the backward form is opt-in in the model (slower there)
    yield kernels
    kernels.LN_FUSED_BWD = prev


def _rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30)).item()


def _fwd_case(M, Kd, seed):
    g = torch.Generator(device='cuda').manual_seed(seed)
    o = (torch.randn(M, Kd, device='cuda', generator=g) * 0.5).bfloat16()
    W = (torch.randn(512, Kd, device='cuda', generator=g) / Kd ** 0.5).bfloat16()
    res = torch.randn(M, 512, device='cuda', generator=g) + 0.3     # non-zero row means
    gamma = 1 + 0.1 * torch.randn(512, device='cuda', generator=g)
    beta = 0.1 * torch.randn(512, device='cuda', generator=g)
    return o, W, res, gamma, beta


@pytest.mark.parametrize('M,Kd', [(4096, 256), (110592, 256), (8192, 1408)])
def test_linear_residual_ln(K, M, Kd):
    o, W, res, gamma, beta = _fwd_case(M, Kd, 1)
    out = K.linear_residual_ln(o, W, res, gamma, beta, 1e-5)
    assert out is not None, 'fused form refused at a fusable shape'
    x1f, x1b, y, mean, rstd = out
    # the residual GEMM part is the unfused kernel's arithmetic (same tile walk, same epilogue sums)
    x1b_ref = torch.empty_like(x1b)
    x1f_ref = K.linear(o, W, residual=res, out_dtype=torch.float32, out2=x1b_ref)
    assert torch.equal(x1f, x1f_ref)
    assert torch.equal(x1b, x1b_ref)
    # LayerNorm of x1f (torch fp32) and the stand-alone kernel
    ref = torch.nn.functional.layer_norm(x1f, (512,), gamma, beta, 1e-5)
    assert _rel(y.float(), ref) < 4e-3
    assert (y.float() - ref).abs().max().item() < 0.05
    mu = x1f.double().mean(1)
    var = x1f.double().var(1, unbiased=False)
    assert ((mean.double() - mu).abs() / (var.sqrt() + 1e-6)).max().item() < 1e-5
    assert ((rstd.double() - (var + 1e-5).rsqrt()).abs() / (var + 1e-5).rsqrt()).max().item() < 1e-5
    yb_un, _, m_un, r_un = K.layernorm_fwd(x1f, gamma, beta, 1e-5)
    assert (y.float() - yb_un.float()).abs().max().item() <= 2 ** -6 * yb_un.float().abs().max().item()
    assert K.ln_fused_status() == 0


def _bwd_case(M, N, seed):
    g = torch.Generator(device='cuda').manual_seed(seed)
    dy = (torch.randn(M, N, device='cuda', generator=g) * 0.1).bfloat16()
    W = (torch.randn(N, 512, device='cuda', generator=g) / N ** 0.5).bfloat16()
    xf = torch.randn(M, 512, device='cuda', generator=g) * 2 + 0.5
    gamma = 1 + 0.1 * torch.randn(512, device='cuda', generator=g)
    mean = xf.mean(1)
    rstd = (xf.var(1, unbiased=False) + 1e-5).rsqrt()
    x = xf.bfloat16()
    dres = torch.randn(M, 512, device='cuda', generator=g)
    return dy, W, x, mean, rstd, gamma, dres


def _ln_bwd_ref(dyl, x, mean, rstd, gamma, dres):
    xh = (x.double() - mean.double()[:, None]) * rstd.double()[:, None]
    gdy = dyl.double() * gamma.double()
    dx = rstd.double()[:, None] * (gdy - gdy.mean(1, keepdim=True) - xh * (gdy * xh).mean(1, keepdim=True))
    return dx + dres.double(), (dyl.double() * xh).sum(0), dyl.double().sum(0)


@pytest.mark.parametrize('M,N,beta', [(4096, 256, False), (110592, 256, False), (16384, 2816, True)])
def test_matmul_nn_ln_bwd(K, M, N, beta):
    dy, W, x, mean, rstd, gamma, dres = _bwd_case(M, N, 2)
    dg = torch.zeros(512, device='cuda')
    db = torch.zeros(512, device='cuda') if beta else None
    out = K.matmul_nn_ln_bwd(dy, W, x, mean, rstd, gamma, dres, dgamma_out=dg, dbeta_out=db)
    assert out is not None, 'fused form refused at a fusable shape'
    dxf, dxb = out
    torch.cuda.synchronize()
    dyl = (dy.float() @ W.float()).bfloat16()          # the unfused GEMM's stored (bf16) output
    dx_ref, dg_ref, db_ref = _ln_bwd_ref(dyl, x, mean, rstd, gamma, dres)
    assert _rel(dxf, dx_ref) < 2e-3
    assert torch.equal(dxb, dxf.bfloat16())
    assert _rel(dg, dg_ref) < 2e-3
    if beta:
        assert _rel(db, db_ref) < 2e-3
    # against the unfused pair (GEMM -> bf16, then the LayerNorm-backward kernel)
    dyk = K.matmul_nn(dy, W)
    dxf_un, _, dg_un, _ = K.layernorm_bwd(dyk, x, mean, rstd, gamma, dres=dres, want_beta=beta)
    assert _rel(dxf, dxf_un) < 1e-3
    assert _rel(dg, dg_un) < 1e-3
    assert K.ln_fused_status() == 0


def test_repeat_bit_identical_and_streams(K):
    """Many launches (fresh epoch each) on two streams: results never change; no timeout."""
    o, W, res, gamma, beta = _fwd_case(4096, 256, 3)
    base = K.linear_residual_ln(o, W, res, gamma, beta, 1e-5)
    side = torch.cuda.Stream()
    for i in range(40):
        st = side if i % 2 else torch.cuda.current_stream()
        with torch.cuda.stream(st):
            again = K.linear_residual_ln(o, W, res, gamma, beta, 1e-5)
        st.synchronize()
        for a, b in zip(again, base):
            assert torch.equal(a, b)
    dy, Wb, x, mean, rstd, gamma2, dres = _bwd_case(4096, 256, 4)
    dg0 = torch.zeros(512, device='cuda')
    b0 = K.matmul_nn_ln_bwd(dy, Wb, x, mean, rstd, gamma2, dres, dgamma_out=dg0)
    for _ in range(20):
        dg = torch.zeros(512, device='cuda')
        b1 = K.matmul_nn_ln_bwd(dy, Wb, x, mean, rstd, gamma2, dres, dgamma_out=dg)
        assert torch.equal(b1[0], b0[0]) and torch.equal(dg, dg0)
    torch.cuda.synchronize()
    assert K.ln_fused_status() == 0


def test_refused_shapes_fall_back(K):
    """Shapes the pair exchange cannot take (M % 2048 != 0) are refused without launching."""
    o, W, res, gamma, beta = _fwd_case(2304, 256, 5)
    assert K.linear_residual_ln(o, W, res, gamma, beta, 1e-5) is None


def test_transformer_layer_fused_vs_unfused(K):
    """A 3D-ViT layer (temporal geometry, B = 8 full size: 110,592 tokens) with the fused
    to_out + residual + LayerNorm forward (and the opt-in fused backward) against the unfused
    kernels: outputs and parameter gradients agree to f32 / bf16 rounding."""
    from ctclip_mi355x import attention as A, functional as Fn
    torch.manual_seed(0)
    tr = A.Transformer(512, depth=1, dim_head=32, heads=8).cuda()
    with torch.no_grad():
        for p in tr.parameters():
            p.add_(0.02 * torch.randn_like(p))
    geo = Fn.Geo(B=8, T=24, Hg=24, Wg=24, heads=8, dim_head=32, mode=1)
    xf0 = torch.randn(geo.M, 512, device='cuda')
    xb0 = xf0.bfloat16()
    dy = torch.randn(geo.M, 512, device='cuda') * 1e-2

    def run(fused, fused_bwd):
        K.LN_FUSED, K.LN_FUSED_BWD = fused, fused_bwd
        for p in tr.parameters():
            p.grad = None
        xf = xf0.clone().requires_grad_(True)
        with K.ln_guard():        # the model uses the fused forms only under a status reader
            yf, yb = tr.run(xf, xb0, geo)
            yf.backward(dy)
        torch.cuda.synchronize()
        return yf.detach(), xf.grad, [p.grad.clone() for p in tr.parameters() if p.grad is not None]

    prev = K.LN_FUSED, K.LN_FUSED_BWD
    try:
        y0, dx0, g0 = run(False, False)
        y1, dx1, g1 = run(True, False)
        y2, dx2, g2 = run(True, True)
    finally:
        K.LN_FUSED, K.LN_FUSED_BWD = prev
    assert _rel(y1, y0) < 2e-3 and _rel(y2, y0) < 2e-3
    assert _rel(dx1, dx0) < 1e-2 and _rel(dx2, dx0) < 1e-2
    for a, b, c in zip(g0, g1, g2):
        assert _rel(b, a) < 2e-2 and _rel(c, a) < 2e-2
    assert K.ln_fused_status() == 0


def test_train_step_raises_on_exchange_timeout(K):
    """Fail loud: a partner tile that never publishes its row statistics (test knob)
    makes the exchange time out.  The trainer's step then (1) is not applied on the device -- the
    status word is the Adam kernel's skip guard, so parameters stay bit-identical -- and (2) raises
    LayerNormExchangeError on the host (train_step two steps later at the latest, check() / flush()
    at once).  A healthy step before it passes the same per-step check."""
    import types
    from ctclip_mi355x.bert import BertConfig
    from ctclip_mi355x.models import build_ctclip, set_finetune_trainable
    from ctclip_mi355x.trainer import CTClipTrainer, LayerNormExchangeError
    torch.manual_seed(0)
    # 2 x 40 x 320 x 320 volumes -> 2 x 4 x 16 x 16 = 2,048 tokens: the fused LayerNorm GEMM's shape
    vit = dict(image_size=320, codebook_size=512, spatial_depth=1, temporal_depth=1)
    bert = BertConfig(vocab_size=1000, hidden_size=768, num_hidden_layers=1, num_attention_heads=12,
                      intermediate_size=3072, max_position_embeddings=64, hidden_dropout_prob=0.0,
                      attention_probs_dropout_prob=0.0)
    model = set_finetune_trainable(build_ctclip(vit, bert)).cuda()
    g = torch.Generator(device='cuda').manual_seed(7)
    hu = torch.randint(-1200, 1201, (2, 1, 40, 320, 320), generator=g, device='cuda', dtype=torch.int32).to(torch.int16)
    ids = torch.randint(5, 1000, (2, 32), generator=g, device='cuda')
    ids[:, 0], ids[:, -1] = 2, 3
    text = types.SimpleNamespace(input_ids=ids, attention_mask=torch.ones_like(ids))
    K.reset_ln_status()
    calls = []
    orig = K.linear_residual_ln

    def spy(*a, **kw):
        out = orig(*a, **kw)
        calls.append(out is not None)
        return out
    K.linear_residual_ln = spy
    tr = CTClipTrainer(model)
    try:
        tr.train_step(text, hu)
        tr.check()                                    # healthy step: checked, no error
        assert calls and all(calls), 'the fused LayerNorm GEMM did not run in the train step'
        assert tr.ln_steps_checked == 1 and K.ln_fused_status() == 0
        before = tr.flat.data.clone()
        m_before = tr.m.clone()
        old = K.set_ln_debug(True, spin_limit=1 << 12)
        try:
            with pytest.raises(LayerNormExchangeError):
                for _ in range(3):                    # raises by the third call at the latest
                    tr.train_step(text, hu)
                tr.check()
        finally:
            K.set_ln_debug(**old)
        torch.cuda.synchronize()
        assert K.ln_fused_status() == 1
        assert torch.equal(tr.flat.data, before) and torch.equal(tr.m, m_before), \
            'a step with a timed-out LayerNorm exchange was applied'
        assert float(tr.flat.grad[:tr.flat.numel].abs().max()) == 0.0   # the dropped step's gradients were cleared
        assert float(tr.flat.status) == 1.0               # this rank's status word, summed (world 1)
    finally:
        K.linear_residual_ln = orig
        K.reset_ln_status()


@pytest.mark.parametrize('nwg,lds_kb', [(16, 80), (64, 80), (200, 100)])
def test_fused_ln_beside_cu_holding_kernels(K, nwg, lds_kb):
    """The LayerNorm-fused GEMM pairs tiles 2k, 2k + 1 on workgroups w, w ^ 8 of one persistent round.
    With other kernels holding CUs (here nwg spinning workgroups, each with enough LDS that no GEMM
    workgroup fits beside it -- as RCCL's resident kernels at N > 1), some GEMM workgroups start only
    when CUs free up; their partners wait (bounded) instead of timing out, and the outputs equal the
    undisturbed launch bit for bit with the status word still 0."""
    from ctclip_mi355x import _lib
    o, W, res, gamma, beta = _fwd_case(110592, 256, 9)
    K.reset_ln_status()
    with K.ln_guard():
        ref = K.linear_residual_ln(o, W, res, gamma, beta, 1e-5)
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    # ~1 ms of spinning at ~2.1 GHz, started first so it holds its CUs when the GEMM dispatches
    with torch.cuda.stream(side):
        _lib.call('ctclip_debug_hold_cus', nwg, 2_000_000, lds_kb * 1024, side.cuda_stream)
    with K.ln_guard():
        out = K.linear_residual_ln(o, W, res, gamma, beta, 1e-5)
    torch.cuda.synchronize()
    assert out is not None
    for a, b in zip(out, ref):
        assert torch.equal(a, b)
    assert K.ln_fused_status() == 0
