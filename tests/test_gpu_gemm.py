"""MFMA GEMM kernel vs a plain torch fp32 reference (GPU)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def K():
    from ctclip_mi355x import kernels
    return kernels


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


@pytest.mark.parametrize('M,N,K_', [(128, 128, 64), (256, 384, 512), (300, 136, 200), (1000, 2816, 512),
                                    (64, 512, 1408), (8, 512, 4096)])
def test_linear_nt(K, M, N, K_):
    torch.manual_seed(0)
    x = torch.randn(M, K_, device='cuda').bfloat16()
    w = torch.randn(N, K_, device='cuda').bfloat16()
    b = torch.randn(N, device='cuda')
    r = torch.randn(M, N, device='cuda')
    y = K.linear(x, w, bias=b, residual=r, out_dtype=torch.float32)
    ref = x.float() @ w.float().t() + b + r
    assert _rel(y, ref) < 1e-5


def test_layout_asymmetric_exact(K):
    # integer-valued operands -> exact f32 results; catches row/col swaps
    M, N, K_ = 256, 256, 128
    x = (torch.arange(M * K_, device='cuda').reshape(M, K_) % 7 - 3).bfloat16()
    w = (torch.arange(N * K_, device='cuda').reshape(N, K_) % 5 - 2).bfloat16()
    y = K.linear(x, w, out_dtype=torch.float32)
    assert torch.equal(y, x.float() @ w.float().t())
    dy = (torch.arange(M * N, device='cuda').reshape(M, N) % 3 - 1).bfloat16()
    dx = K.matmul_nn(dy, w, out_dtype=torch.float32)
    assert torch.equal(dx, dy.float() @ w.float())
    dw = K.matmul_tn(dy, x, split_k=1)
    assert torch.equal(dw, dy.float().t() @ x.float())
    dw2 = K.matmul_tn(dy, x, split_k=3)
    assert torch.equal(dw2, dy.float().t() @ x.float())


@pytest.mark.parametrize('M,N,K_', [(512, 512, 256), (1000, 1408, 512), (4096, 512, 2816)])
def test_matmul_nn(K, M, N, K_):
    torch.manual_seed(1)
    dy = torch.randn(M, N, device='cuda').bfloat16()
    w = torch.randn(N, K_, device='cuda').bfloat16()
    dx = K.matmul_nn(dy, w, out_dtype=torch.float32)
    assert _rel(dx, dy.float() @ w.float()) < 1e-5


@pytest.mark.parametrize('M,N,K_', [(4096, 512, 512), (20000, 256, 512), (1024, 2816, 512), (8, 512, 1024)])
def test_matmul_tn(K, M, N, K_):
    torch.manual_seed(2)
    dy = torch.randn(M, N, device='cuda').bfloat16()
    x = torch.randn(M, K_, device='cuda').bfloat16()
    dw = K.matmul_tn(dy, x)
    assert _rel(dw, dy.float().t() @ x.float()) < 1e-5


@pytest.mark.parametrize('M', [384, 40000])    # 128-tile kernel / 256-tile glds kernel
def test_gelu_and_geglu_epilogue(K, M):
    torch.manual_seed(3)
    Kd, N = 512, 1024
    x = torch.randn(M, Kd, device='cuda').bfloat16()
    w = (torch.randn(N, Kd, device='cuda') / 20).bfloat16()
    pre = torch.empty(M, N, device='cuda', dtype=torch.bfloat16)
    y = K.linear(x, w, act=K.ACT_GELU, out2=pre)
    ref_pre = x.float() @ w.float().t()
    assert _rel(y, torch.nn.functional.gelu(ref_pre)) < 4e-3
    assert _rel(pre, ref_pre) < 4e-3
    g = torch.empty(M, N // 2, device='cuda', dtype=torch.bfloat16)
    h = K.linear(x, w, act=K.ACT_GEGLU, out2=g)
    hf = h.float().reshape(M, N // 64, 2, 32)
    ref_g = (torch.nn.functional.gelu(hf[:, :, 1]) * hf[:, :, 0]).reshape(M, N // 2)
    assert _rel(g, ref_g) < 4e-3
    assert _rel(h, ref_pre) < 4e-3


@pytest.mark.parametrize('M,N,K_,lay', [(8192, 2816, 512, 'nt'), (4096, 512, 1408, 'nt'), (20480, 512, 512, 'nn'),
                                        (20480, 512, 2816, 'nn'), (40960, 2816, 512, 'tn'), (65536, 512, 256, 'tn')])
def test_large_tile_layouts(K, M, N, K_, lay):
    """Shapes that dispatch to the 256x256 glds kernel (all three layouts, residual/bias epilogues)."""
    torch.manual_seed(7)
    if lay == 'nt':
        x = torch.randn(M, K_, device='cuda').bfloat16()
        w = torch.randn(N, K_, device='cuda').bfloat16()
        r = torch.randn(M, N, device='cuda')
        b = torch.randn(N, device='cuda')
        y = K.linear(x, w, bias=b, residual=r, out_dtype=torch.float32)
        assert _rel(y, x.float() @ w.float().t() + b + r) < 1e-5
    elif lay == 'nn':
        dy = torch.randn(M, N, device='cuda').bfloat16()
        w = torch.randn(N, K_, device='cuda').bfloat16()
        dx = K.matmul_nn(dy, w, out_dtype=torch.float32)
        assert _rel(dx, dy.float() @ w.float()) < 1e-5
    else:
        dy = torch.randn(M, N, device='cuda').bfloat16()
        x = torch.randn(M, K_, device='cuda').bfloat16()
        dw = K.matmul_tn(dy, x)
        assert _rel(dw, dy.float().t() @ x.float()) < 1e-5


def test_large_tile_exact_asymmetric(K):
    M, N, K_ = 1024, 1024, 256
    x = (torch.arange(M * K_, device='cuda').reshape(M, K_) % 7 - 3).bfloat16()
    w = (torch.arange(N * K_, device='cuda').reshape(N, K_) % 5 - 2).bfloat16()
    y = K.linear(x, w, out_dtype=torch.float32)
    assert torch.equal(y, x.float() @ w.float().t())
    dy = (torch.arange(M * N, device='cuda').reshape(M, N) % 3 - 1).bfloat16()
    dx = K.matmul_nn(dy, w, out_dtype=torch.float32)
    assert torch.equal(dx, dy.float() @ w.float())
    dw = K.matmul_tn(dy, x, split_k=8)
    assert torch.equal(dw, dy.float().t() @ x.float())


@pytest.mark.parametrize('M', [1000, 70000])
def test_argmax_epilogue(K, M):
    torch.manual_seed(4)
    Nc, Kd = 1024, 512
    x = torch.randn(M, Kd, device='cuda').bfloat16()
    w = torch.randn(Nc, Kd, device='cuda').bfloat16()
    nt = Nc // 64
    out = torch.empty(M, nt, 2, device='cuda', dtype=torch.float32)
    K.gemm_raw(M, Nc, Kd, x, Kd, True, w, Kd, True, out, nt, act=K.ACT_ARGMAX)
    vals = out[..., 0]
    idx = out[..., 1].contiguous().view(torch.int32)
    s = x.float() @ w.float().t()
    best = vals.argmax(1)
    got = idx.gather(1, best[:, None])[:, 0].long()
    ref = s.argmax(1)
    assert (got == ref).float().mean().item() > 0.999


@pytest.mark.parametrize('M,N,K_,act', [(1024, 2304, 768, 0), (1024, 3072, 768, 1), (1024, 768, 3072, 0),
                                        (300, 136, 200, 0)])
def test_linear_split_weight(K, M, N, K_, act):
    """Text-tower GEMMs on hi / lo split weights (gemm.hip B2, kernels.cast_bf16_split): the f32
    weight seen to ~16 mantissa bits, so against an f32 matmul with the SAME bf16 activations the
    error is the f32-accumulation level, far below one bf16 rounding of the weight.  Covers the
    split-K combine path (K = 3072, M = 1024) and ragged edges."""
    torch.manual_seed(5)
    x = torch.randn(M, K_, device='cuda').bfloat16()
    W = torch.randn(N, K_, device='cuda') * 0.05
    b = torch.randn(N, device='cuda')
    hi, lo = K.cast_bf16_split(W)
    assert torch.equal(hi, W.bfloat16()) and torch.equal(lo, (W - hi.float()).bfloat16())
    pre = torch.empty(M, N, device='cuda', dtype=torch.bfloat16) if act else None
    y = K.linear(x, hi, bias=b, out_dtype=torch.float32, w_lo=lo, act=act, out2=pre)
    ref = x.float() @ W.t() + b
    if act:
        assert _rel(pre, ref) < 4e-3          # bf16 pre-activation copy
        ref = torch.nn.functional.gelu(ref)
    e_split = _rel(y, ref)
    e_hi = _rel(K.linear(x, hi, bias=b, out_dtype=torch.float32, act=act,
                         out2=torch.empty_like(pre) if act else None), ref)
    print(f'split {e_split:.2e}  hi-only {e_hi:.2e}')
    assert e_split < 2e-5 and e_hi > 20 * e_split


def test_adam_writes_split_shadow(K):
    """The Adam pass writes hi = bf16(p) and lo = bf16(p - hi) of the UPDATED parameter."""
    torch.manual_seed(6)
    n = 100003
    p, g = torch.randn(n, device='cuda'), torch.randn(n, device='cuda')
    m, v = torch.zeros(n, device='cuda'), torch.zeros(n, device='cuda')
    hi = torch.empty(n, device='cuda', dtype=torch.bfloat16)
    lo = torch.empty_like(hi)
    K.adam(p[1:], g[1:], m[1:], v[1:], lr=1e-3, b1=0.9, b2=0.99, eps=1e-8, wd=0.0, step=1, p_bf16=hi[1:],
           p_bf16_lo=lo[1:])
    torch.cuda.synchronize()
    assert torch.equal(hi[1:], p[1:].bfloat16())
    assert torch.equal(lo[1:], (p[1:] - hi[1:].float()).bfloat16())




@pytest.mark.parametrize('M,N,K_', [(8, 512, 294912), (2, 512, 294912), (16, 128, 4096), (5, 64, 256 * 7)])
def test_skinny_linear(K, M, N, K_):
    """The HBM-streaming skinny GEMM of the image projection (to_visual_latent, ct_clip/ct_clip.py:
    564,767; csrc/proj.hip) against an f64 matmul of the same bf16 operands, integer-exact data for
    the layout (a row / column / k-permutation slip cannot pass), and deterministic repeats."""
    torch.manual_seed(4)
    x = torch.randn(M, K_, device='cuda').bfloat16()
    w = (torch.randn(N, K_, device='cuda') * 0.01).bfloat16()
    y = K.skinny_linear(x, w)
    assert y is not None
    ref = (x.double() @ w.double().t())
    assert _rel(y, ref) < 1e-5
    assert torch.equal(K.skinny_linear(x, w), y)
    xi = (torch.arange(M * K_, device='cuda').reshape(M, K_) % 5 - 2).bfloat16()
    wi = ((torch.arange(N * K_, device='cuda').reshape(N, K_) * 7) % 3 - 1).bfloat16()
    if K_ <= 4096:      # sums stay exact in f32
        assert torch.equal(K.skinny_linear(xi, wi), (xi.double() @ wi.double().t()).float())
    assert K.skinny_linear(torch.zeros(17, K_, device='cuda').bfloat16(), w) is None


@pytest.mark.parametrize('M,N,K_', [(8, 512, 294912), (3, 128, 128 * 5)])
def test_skinny_linear_f32(K, M, N, K_):
    """The f32 twin (ctclip_skinny_sgemm: the precise image towers' projection): f32 accuracy against
    f64 (an f32 fma per product, f32 slabs), integer-exact data for the k layout, deterministic."""
    torch.manual_seed(5)
    x = torch.randn(M, K_, device='cuda')
    w = torch.randn(N, K_, device='cuda') * 0.01
    y = K.skinny_linear(x, w)
    assert y is not None and y.dtype == torch.float32
    assert _rel(y, x.double() @ w.double().t()) < 1e-6
    assert torch.equal(K.skinny_linear(x, w), y)
    xi = (torch.arange(M * K_, device='cuda').reshape(M, K_) % 5 - 2).float()
    wi = ((torch.arange(N * K_, device='cuda').reshape(N, K_) * 7) % 3 - 1).float()
    assert torch.equal(K.skinny_linear(xi, wi), (xi.double() @ wi.double().t()).float())
    assert K.skinny_linear(x[:, :K_ - 4], w[:, :K_ - 4]) is None     # K % 128 != 0
