"""Large-tile MFMA GEMM paths (gemm256.hip) at shapes that dispatch to them (>= 160 tiles of
256 x 256): every layout and fused epilogue vs a plain torch fp32 reference, and the 8-phase
256x256x64 kernel bit-identical to the 128x256x32 kernel (same MFMA k-order per accumulator)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def K():
    from ctclip_mi355x import kernels
    return kernels


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


def _variants(K, fn):
    """Outputs of the 8-phase kernel (persistent, key 8) and the 128x256x32 kernel (key 1); the
    8-phase kernel with one workgroup per tile, persistent on a grid capped at 92 workgroups, and
    with its bf16 / GEGLU epilogue stores re-laid through LDS (ctclip_gemm_set_epi_lds), must match
    the persistent one bit for bit."""
    from ctclip_mi355x import _lib
    outs = {}
    lib = _lib.lib()
    prev, prev_p = lib.ctclip_gemm_set_variant(8), lib.ctclip_gemm_set_persist(1)
    prev_l = lib.ctclip_gemm_set_epi_lds(0)
    snap = lambda o: o.clone() if torch.is_tensor(o) else o  # noqa: E731
    try:
        lib.ctclip_gemm_set_epi_lds(1)
        lds = snap(fn())
        torch.cuda.synchronize()
        lib.ctclip_gemm_set_epi_lds(2)      # the same with L2-dropping (sc1) stores
        lds_sc1 = snap(fn())
        torch.cuda.synchronize()
        lib.ctclip_gemm_set_epi_lds(3)      # direct stores, sc1
        sc1 = snap(fn())
        torch.cuda.synchronize()
        lib.ctclip_gemm_set_epi_lds(0)
        for v in (8, 1):
            lib.ctclip_gemm_set_variant(v)
            outs[v] = snap(fn())
            torch.cuda.synchronize()
        lib.ctclip_gemm_set_variant(8)
        lib.ctclip_gemm_set_grid_cap(92)      # persistent walk on a capped grid (two-stream sharing)
        capped = snap(fn())
        torch.cuda.synchronize()
        lib.ctclip_gemm_set_grid_cap(0)
        lib.ctclip_gemm_set_persist(0)
        single = snap(fn())
        torch.cuda.synchronize()
    finally:
        lib.ctclip_gemm_set_grid_cap(0)
        lib.ctclip_gemm_set_variant(prev)
        lib.ctclip_gemm_set_persist(prev_p if prev_p >= 0 else 1)
        lib.ctclip_gemm_set_epi_lds(max(prev_l, 0))
    if torch.is_tensor(single):
        assert torch.equal(lds, outs[8]), 'LDS-relaid epilogue stores differ'
        assert torch.equal(lds_sc1, outs[8]), 'LDS-relaid sc1 epilogue stores differ'
        assert torch.equal(sc1, outs[8]), 'sc1 epilogue stores differ'
        assert torch.equal(single, outs[8]), 'persistent 8-phase GEMM differs from one workgroup per tile'
        assert torch.equal(capped, outs[8]), 'persistent 8-phase GEMM on a capped grid differs'
    return outs


def _raw(K, M, N, Kd, A, lda, ak, B, ldb, bk, C, ldc, **kw):
    K._gemm_raw(M, N, Kd, A, lda, ak, B, ldb, bk, C, ldc, **kw)
    return C


@pytest.mark.parametrize('M,N,Kd', [(4000, 2816, 512), (8192, 1536, 1408), (5000, 2048, 192), (9000, 2816, 512)])
def test_nt_bias_residual(K, M, N, Kd):
    torch.manual_seed(0)
    x = torch.randn(M, Kd, device='cuda').bfloat16()
    w = torch.randn(N, Kd, device='cuda').bfloat16()
    b = torch.randn(N, device='cuda')
    r = torch.randn(M, N, device='cuda')
    outs = _variants(K, lambda: K.linear(x, w, bias=b, residual=r, out_dtype=torch.float32))
    ref = x.float() @ w.float().t() + b + r
    assert _rel(outs[8], ref) < 1e-5
    assert torch.equal(outs[8], outs[1])


@pytest.mark.parametrize('M,N,Kd,ak', [(110592 // 8, 512, 256, True), (5000, 768, 512, True), (9000, 512, 512, False)])
def test_residual_f32_with_bf16_shadow(K, M, N, Kd, ak):
    """The residual epilogue (f32 out = acc + R, bf16 shadow in C2; gemm256.hip LM -2): full and
    ragged tiles, both A layouts; the shadow is the f32 output rounded to bf16, bit for bit."""
    torch.manual_seed(1)
    x = torch.randn(M, Kd, device='cuda').bfloat16()
    w = torch.randn(N, Kd, device='cuda').bfloat16()
    r = torch.randn(M, N, device='cuda')
    out = torch.empty(M, N, device='cuda')
    sh = torch.empty(M, N, device='cuda', dtype=torch.bfloat16)
    if ak:
        K.linear(x, w, residual=r, out_dtype=torch.float32, out=out, out2=sh)
    else:
        xt = x.t().contiguous()      # A stored M-contiguous (the dW-style layout)
        K._gemm_raw(M, N, Kd, xt, M, False, w, Kd, True, out, N, R=r, ldr=N, C2=sh, ldc2=N)
    ref = x.float() @ w.float().t() + r
    assert _rel(out, ref) < 1e-5
    assert torch.equal(sh, out.bfloat16())


@pytest.mark.parametrize('ak,bk', [(True, False), (False, True), (False, False)])
def test_layouts(K, ak, bk):
    torch.manual_seed(1)
    M, N, Kd = 3000, 3328, 704
    A = torch.randn(M, Kd, device='cuda').bfloat16()
    B = torch.randn(N, Kd, device='cuda').bfloat16()
    Am = A if ak else A.t().contiguous()
    Bm = B if bk else B.t().contiguous()

    def run():
        C = torch.empty(M, N, device='cuda', dtype=torch.float32)
        return _raw(K, M, N, Kd, Am, Am.stride(0), ak, Bm, Bm.stride(0), bk, C, N)
    outs = _variants(K, run)
    ref = A.float() @ B.float().t()
    assert _rel(outs[8], ref) < 1e-5
    assert torch.equal(outs[8], outs[1])


def test_tn_split_slabs(K):
    torch.manual_seed(2)
    M, N, Kd = 65536, 512, 512          # dW[N, Kd] = dy^T x over 65536 tokens
    dy = torch.randn(M, N, device='cuda').bfloat16()
    x = torch.randn(M, Kd, device='cuda').bfloat16()
    outs = _variants(K, lambda: K.matmul_tn(dy, x, split_k=40))
    ref = dy.float().t() @ x.float()
    assert _rel(outs[8], ref) < 1e-5
    assert torch.allclose(outs[8], outs[1], rtol=0, atol=1e-3)


@pytest.mark.parametrize('N,Kd,cols,packed', [(2816, 512, 512, True), (512, 1408, 1365, False)])
def test_tn_slabs_into_unpacked_rows(K, N, Kd, cols, packed):
    """The FeedForward weight gradients at the step's token count: the split-K slabs reduced
    straight into the unpacked, accumulated .grad rows (ctclip_reduce_slabs_rows; W1's GEGLU-packed
    rows through ff1_rowmap, W2's padded columns cropped) equal dW followed by unpack_rows, bit for
    bit."""
    from ctclip_mi355x import functional as Fn
    torch.manual_seed(3)
    M = 110592
    dy = (torch.randn(M, N, device='cuda') * 0.1).bfloat16()
    x = (torch.randn(M, Kd, device='cuda') * 0.1).bfloat16()
    rowmap = Fn.ff1_rowmap(1365, dy.device) if packed else None
    rows = 2730 if packed else N
    base = torch.randn(rows, cols, device='cuda')
    fused, ref = base.clone(), base.clone()
    K.matmul_tn(dy, x, unpack=(fused, rowmap, cols))
    dw = K.matmul_tn(dy, x)
    K.unpack_rows(dw, ref, rowmap=rowmap, cols=cols, accumulate=True)
    torch.cuda.synchronize()
    assert torch.equal(fused, ref)
    full = dy.float().t() @ x.float()
    want = base.clone()
    if packed:
        keep = rowmap >= 0
        want.index_add_(0, rowmap[keep].long(), full[keep][:, :cols])
    else:
        want += full[:, :cols]
    assert _rel(fused - base, want - base) < 1e-5


def test_nn_accumulate_shadow(K):
    torch.manual_seed(3)
    M, N, Kd = 10000, 2816, 1024
    dy = torch.randn(M, N, device='cuda').bfloat16()
    w = torch.randn(N, Kd, device='cuda').bfloat16()
    base = torch.randn(M, Kd, device='cuda')

    def run():
        C = base.clone()
        return K.matmul_nn(dy, w, out=C, accumulate=True)
    outs = _variants(K, run)
    ref = base + dy.float() @ w.float()
    assert _rel(outs[8], ref) < 1e-5
    assert torch.equal(outs[8], outs[1])


def test_geglu_and_gelu(K):
    torch.manual_seed(4)
    M, N, Kd = 6000, 2816, 512
    x = torch.randn(M, Kd, device='cuda').bfloat16()
    w = (torch.randn(N, Kd, device='cuda') * 0.05).bfloat16()

    def geglu():
        g = torch.empty(M, N // 2, device='cuda', dtype=torch.bfloat16)
        h = K.linear(x, w, act=K.ACT_GEGLU, out2=g)
        return torch.cat([h.float(), g.float()], 1)
    outs = _variants(K, geglu)
    h = (x.float() @ w.float().t()).bfloat16().float()
    hv = h.view(M, N // 64, 2, 32)
    g = (torch.nn.functional.gelu(hv[:, :, 1]) * hv[:, :, 0]).reshape(M, N // 2)
    assert _rel(outs[8][:, :N], h) < 1e-2
    assert _rel(outs[8][:, N:], g) < 1e-2
    assert torch.equal(outs[8], outs[1])

    def gelu():
        pre = torch.empty(M, N, device='cuda', dtype=torch.bfloat16)
        y = K.linear(x, w, act=K.ACT_GELU, out2=pre)
        return torch.cat([y.float(), pre.float()], 1)
    o2 = _variants(K, gelu)
    pre = x.float() @ w.float().t()
    assert _rel(o2[8][:, :N], torch.nn.functional.gelu(pre)) < 1e-2
    assert torch.equal(o2[8], o2[1])


def test_batched_argmax(K):
    torch.manual_seed(5)
    nb, M, N, Kd = 2, 4096, 2560, 512
    A = torch.randn(nb, M, Kd, device='cuda').bfloat16()
    B = torch.randn(N, Kd, device='cuda').bfloat16()

    def run():
        C = torch.empty(nb, M, N // 64, 2, device='cuda', dtype=torch.float32)
        K._gemm_raw(M, N, Kd, A, Kd, True, B, Kd, True, C, N // 64, act=K.ACT_ARGMAX if hasattr(K, 'ACT_ARGMAX')
                    else 3, batch=nb, sA=M * Kd, sB=0, sC=M * (N // 64))
        return C
    outs = _variants(K, run)
    assert torch.equal(outs[8], outs[1])
    ref = (A.float() @ B.float().t()).view(nb, M, N // 64, 64)
    idx = outs[8][..., 1].view(torch.int32).long()
    best = ref.argmax(-1) + torch.arange(N // 64, device='cuda') * 64
    agree = (idx == best).float().mean().item()
    assert agree > 0.999, agree


@pytest.mark.parametrize('M', [6000, 300])     # 8-phase kernel / 128-tile kernel
def test_geglu_bwd_fused(K, M):
    """act 4: dh = geglu_bwd(dy . W2p, h) in one GEMM == the two-kernel path, bit for bit."""
    torch.manual_seed(6)
    D, G = 512, 1408
    dy = (torch.randn(M, D, device='cuda') * 0.1).bfloat16()
    w2p = (torch.randn(D, G, device='cuda') * 0.05).bfloat16()
    h = torch.randn(M, 2 * G, device='cuda').bfloat16()
    fused = K.matmul_nn_geglu_bwd(dy, w2p, h)
    ref = K.geglu_bwd(K.matmul_nn(dy, w2p), h)
    if M >= 1024:
        assert torch.equal(fused, ref)
    else:   # the stand-alone small GEMM runs split-K (different f32 summation order)
        assert _rel(fused, ref) < 5e-3
    # and against torch fp32 math on the bf16-rounded dg
    dg = (dy.float() @ w2p.float()).bfloat16().float()
    hv = h.float().view(M, G // 32, 2, 32)
    x, gt = hv[:, :, 0], hv[:, :, 1]
    d = dg.view(M, G // 32, 32)
    cdf = 0.5 * (1 + torch.erf(gt / 2 ** 0.5))
    pdf = torch.exp(-0.5 * gt * gt) / (2 * torch.pi) ** 0.5
    ox = d * torch.nn.functional.gelu(gt)
    og = d * x * (cdf + gt * pdf)
    refm = torch.stack([ox, og], 2).reshape(M, 2 * G)
    assert _rel(fused, refm) < 1e-2


@pytest.mark.parametrize('M,N,n2', [(41000, 256, 256), (45000, 512, 256), (1000, 512, 256)])
def test_l2norm_epilogue(K, M, N, n2):
    """act 5 (gemm256.hip epilogue_t<6>, and the GEMM + l2n kernel pair for small shapes): q equals
    the plain GEMM bit for bit, q_n = per 32-column head l2norm(q) * scale equals the stand-alone
    l2norm kernel's bit for bit (same summation order); ragged M, N > n2 (the KV case)."""
    torch.manual_seed(9)
    x = torch.randn(M, 512, device='cuda').bfloat16()
    w = (torch.randn(N, 512, device='cuda') * 0.05).bfloat16()
    sc = torch.rand(32, device='cuda') + 0.5
    qn = torch.empty(M, n2, device='cuda', dtype=torch.bfloat16)
    q = K.linear(x, w, out2=qn, l2n_scale=sc, l2n_cols=n2)
    q_ref = K.linear(x, w)
    if M >= 40960:
        assert torch.equal(q, q_ref)
    else:   # the plain small GEMM splits K (python _auto_split); act 5 runs unsplit
        assert _rel(q, q_ref) < 4e-3
    qn_ref = K.l2norm_scale_fwd(q[:, :n2], n2 // 32, 32, sc)
    assert torch.equal(qn, qn_ref)
