"""BERT train-mode dropout (transformers BertEmbeddings / BertSelfAttention / BertSelfOutput /
BertOutput, p = 0.1 in the reference's train step, ct_clip/ct_clip.py:685-686): the hidden-state
kernel (ctclip_dropout) and the attention-probability dropout inside the fused attention kernels,
against torch references that regenerate the same hash mask (splitmix64 finaliser of
seed ^ index * golden ratio, kept iff the low 32 bits >= p * 2^32)."""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
dev = 'cuda'
GOLD, C1, C2 = 0x9E3779B97F4A7C15, 0xff51afd7ed558ccd, 0xc4ceb9fe1a85ec53


def s64(c):
    c &= 2 ** 64 - 1
    return c - 2 ** 64 if c >= 2 ** 63 else c


def keep_mask(idx, seed, p):
    """idx int64 tensor -> bool keep mask (uint64 arithmetic emulated in wrapping int64)."""
    x = torch.bitwise_xor(idx * s64(GOLD), torch.full_like(idx, s64(seed)))
    for c in (C1, C2):
        x = x ^ ((x >> 33) & ((1 << 31) - 1))
        x = x * s64(c)
    x = x ^ ((x >> 33) & ((1 << 31) - 1))
    thresh = int(min(4294967295.0, float(np.float32(p)) * 4294967296.0))
    return (x & 0xffffffff) >= thresh


@pytest.fixture(scope='module')
def K():
    from ctclip_mi355x import kernels
    return kernels


def rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def test_hidden_dropout(K):
    torch.manual_seed(0)
    n = 1024 * 768
    x = torch.randn(1024, 768, device=dev)
    r = torch.randn(1024, 768, device=dev)
    p, seed = 0.1, 0x1234_5678_9abc_def0
    yf, yb = K.dropout(x, p, seed, res=r, out_bf16=True)
    keep = keep_mask(torch.arange(n, device=dev), seed, p).view(1024, 768)
    scale = np.float32(1.0) / (np.float32(1.0) - np.float32(p))
    ref = torch.where(keep, x * float(scale), torch.zeros_like(x)) + r
    assert torch.equal(yf, ref)
    assert torch.equal(yb, ref.bfloat16())
    assert abs(keep.float().mean().item() - (1 - p)) < 3e-3
    # backward = same call on the gradient: same mask
    g, _ = K.dropout(torch.ones_like(x), p, seed)
    assert torch.equal(g != 0, keep)
    # a different seed gives a different mask
    g2, _ = K.dropout(torch.ones_like(x), p, seed + 1)
    assert (g2 != g).float().mean().item() > 0.1


def test_attention_prob_dropout_fwd_bwd(K):
    """BERT shape (L = 128, 12 heads x 64, ragged key mask): O, dQ, dK, dV against torch autograd
    on softmax(QK^T/8 + mask) * keep / (1 - p) . V with the regenerated mask (bf16 tolerance)."""
    torch.manual_seed(1)
    B, L, H, D = 2, 128, 12, 64
    p, seed = 0.1, 987654321
    qkv = torch.randn(B * L, 3 * H * D, device=dev).bfloat16()
    lens = [128, 77]
    kmask = torch.zeros(B, L, dtype=torch.int32, device=dev)
    for b, n in enumerate(lens):
        kmask[b, :n] = 1
    q, k, v = qkv[:, :H * D], qkv[:, H * D:2 * H * D], qkv[:, 2 * H * D:]
    scale = 1.0 / math.sqrt(D)
    o, lse = K.attn_fwd(q, k, v, L=L, H=H, D=D, nseq=B, scale=scale, seq=(1, L, 0, 1), kmask=kmask,
                        dropout=(p, seed))
    dout = torch.randn(B * L, H * D, device=dev).bfloat16()
    dq, dk, dv = (torch.empty(B * L, H * D, device=dev, dtype=torch.bfloat16) for _ in range(3))
    K.attn_bwd(q, k, v, o, lse, dout, dq, dk, dv, L=L, H=H, D=D, nseq=B, scale=scale, seq=(1, L, 0, 1),
               kmask=kmask, dropout=(p, seed))
    # torch reference
    qr, kr, vr = (t.float().view(B, L, H, D).transpose(1, 2).requires_grad_(True) for t in (q, k, v))
    s = qr @ kr.transpose(-1, -2) * scale
    s = s.masked_fill(kmask[:, None, None, :] == 0, float('-inf'))
    P = torch.softmax(s, -1)
    idx = (((torch.arange(B, device=dev)[:, None, None, None] * H + torch.arange(H, device=dev)[None, :, None, None])
            * L + torch.arange(L, device=dev)[None, None, :, None]) * L + torch.arange(L, device=dev)[None, None, None, :])
    keep = keep_mask(idx, seed, p)
    dscale = float(np.float32(1.0) / (np.float32(1.0) - np.float32(p)))
    O = (P * keep * dscale) @ vr
    O.backward(dout.float().view(B, L, H, D).transpose(1, 2))
    Oref = O.detach().transpose(1, 2).reshape(B * L, H * D)
    assert rel(o, Oref) < 1e-2
    for got, ref in ((dq, qr.grad), (dk, kr.grad), (dv, vr.grad)):
        assert rel(got, ref.transpose(1, 2).reshape(B * L, H * D)) < 2e-2
    # p = 0 path unchanged
    o0, _ = K.attn_fwd(q, k, v, L=L, H=H, D=D, nseq=B, scale=scale, seq=(1, L, 0, 1), kmask=kmask)
    O0 = (P.detach() @ vr.detach()).transpose(1, 2).reshape(B * L, H * D)
    assert rel(o0, O0) < 1e-2 and rel(o, o0) > 0.05


def test_bert_train_step_with_dropout(K):
    """Whole BERT layer stack in train mode with p = 0.1: finite, differs from eval, masks
    regenerated consistently (two forwards with the same call counter give the same output)."""
    from ctclip_mi355x.bert import BertModel, BertConfig
    torch.manual_seed(2)
    m = BertModel(BertConfig(vocab_size=1000, hidden_size=768, num_hidden_layers=2, num_attention_heads=12,
                             intermediate_size=3072, max_position_embeddings=128)).cuda()
    ids = torch.randint(5, 1000, (2, 64), device=dev)
    mask = torch.ones_like(ids)
    m.eval()
    with torch.no_grad():
        ye = m(ids, mask)[0].clone()
    m.train()
    m._drop_calls = 10
    y1 = m(ids, mask)[0]
    m._drop_calls = 10
    y2 = m(ids, mask)[0]
    torch.cuda.synchronize()
    assert torch.equal(y1, y2)
    assert torch.isfinite(y1).all() and rel(y1, ye) > 0.05
    y1[:, 0].float().square().sum().backward()
    g = m.encoder.layer[0].attention.self.query.weight.grad
    assert g is not None and torch.isfinite(g).all() and g.abs().sum().item() > 0


def test_bert_layer_dropout_grads_match_torch(K):
    """BertLayerFn with all three in-layer dropout sites on (attention probabilities, attention
    output, FF output; p = 0.1): output, dx and every weight / bias / LN gradient against torch
    autograd in fp32 on the same masked graph, masks regenerated from the per-site seeds
    (transformers BertLayer, the reference's text tower, ct_clip/ct_clip.py:685-686)."""
    from ctclip_mi355x import functional as Fn
    torch.manual_seed(3)
    B, L, H, D, I = 2, 64, 12, 64, 3072
    Hd = H * D
    p, s_attn, s_out1, s_out2 = 0.1, 0x1111_2222_3333_4444, 0x5555_6666_7777_8888, 0x0123_4567_89ab_cdef
    eps = 1e-12

    def prm(*shape, scale=0.03):
        return torch.nn.Parameter((torch.randn(*shape, device=dev) * scale).bfloat16().float())

    Wq, Wk, Wv, Wo = prm(Hd, Hd), prm(Hd, Hd), prm(Hd, Hd), prm(Hd, Hd)
    bq, bk, bv, bo = prm(Hd), prm(Hd), prm(Hd), prm(Hd)
    Wi, bi, Wout, bout = prm(I, Hd), prm(I), prm(Hd, I), prm(Hd)
    ln1_w, ln1_b = torch.nn.Parameter(1 + 0.1 * torch.randn(Hd, device=dev)), prm(Hd)
    ln2_w, ln2_b = torch.nn.Parameter(1 + 0.1 * torch.randn(Hd, device=dev)), prm(Hd)
    params = [Wq, bq, Wk, bk, Wv, bv, Wo, bo, ln1_w, ln1_b, Wi, bi, Wout, bout, ln2_w, ln2_b]
    x = torch.randn(B * L, Hd, device=dev).bfloat16().float().requires_grad_(True)
    lens = [64, 41]
    kmask = torch.zeros(B, L, dtype=torch.int32, device=dev)
    for b, n in enumerate(lens):
        kmask[b, :n] = 1
    R = torch.randn(B * L, Hd, device=dev)

    yf, _ = Fn.BertLayerFn.apply(x, x.detach().bfloat16(), kmask, B, L, H, eps, *params,
                                 (p, p, s_attn, s_out1, s_out2))
    (yf * R).sum().backward()
    got = [x.grad.clone()] + [q.grad.clone() for q in params]
    for t in [x] + params:
        t.grad = None

    # torch fp32 reference on the same masks
    dscale = float(np.float32(1.0) / (np.float32(1.0) - np.float32(p)))
    n_h = torch.arange(B * L * Hd, device=dev)
    keep1 = keep_mask(n_h, s_out1, p).view(B * L, Hd)
    keep2 = keep_mask(n_h, s_out2, p).view(B * L, Hd)
    idx = (((torch.arange(B, device=dev)[:, None, None, None] * H + torch.arange(H, device=dev)[None, :, None, None])
            * L + torch.arange(L, device=dev)[None, None, :, None]) * L + torch.arange(L, device=dev)[None, None, None, :])
    keepa = keep_mask(idx, s_attn, p)
    heads = lambda t: t.view(B, L, H, D).transpose(1, 2)  # noqa: E731
    q, k, v = heads(x @ Wq.t() + bq), heads(x @ Wk.t() + bk), heads(x @ Wv.t() + bv)
    s = (q @ k.transpose(-1, -2)) / math.sqrt(D)
    s = s.masked_fill(kmask[:, None, None, :] == 0, float('-inf'))
    P = torch.softmax(s, -1) * keepa * dscale
    ctxv = (P @ v).transpose(1, 2).reshape(B * L, Hd)
    a = (ctxv @ Wo.t() + bo) * keep1 * dscale + x
    x1 = torch.nn.functional.layer_norm(a, (Hd,), ln1_w, ln1_b, eps)
    h = torch.nn.functional.gelu(x1 @ Wi.t() + bi)
    b2 = (h @ Wout.t() + bout) * keep2 * dscale + x1
    y = torch.nn.functional.layer_norm(b2, (Hd,), ln2_w, ln2_b, eps)
    (y * R).sum().backward()
    ref = [x.grad] + [q.grad for q in params]
    assert rel(yf, y.detach()) < 2e-2
    names = ['x', 'Wq', 'bq', 'Wk', 'bk', 'Wv', 'bv', 'Wo', 'bo', 'ln1_w', 'ln1_b', 'Wi', 'bi', 'Wout', 'bout',
             'ln2_w', 'ln2_b']
    errs = {n: rel(g_, r_) for n, g_, r_ in zip(names, got, ref)}
    print('BertLayerFn dropout grads rel err: ' + ', '.join(f'{n} {e:.1e}' for n, e in errs.items()))
    for n, e in errs.items():
        if n == 'bk':    # exactly 0 in exact arithmetic (softmax is shift-invariant per query row)
            continue
        assert e < 5e-2, (n, e)
    # the key bias gradient: both sides are rounding noise around 0, far below the query bias's
    assert got[names.index("bk")].norm() < 3e-2 * got[names.index("bq")].norm()


def test_dropout_fused_into_split_k_combine(K):
    """linear(..., dropout=(p, seed)) (BertSelfOutput / BertOutput dense -> dropout -> + input): the
    mask applied in the split-K combine equals the stand-alone kernel bit for bit."""
    torch.manual_seed(3)
    M, N, Kd = 1024, 768, 3072
    x = (torch.randn(M, Kd, device=dev) * 0.5).bfloat16()
    W = (torch.randn(N, Kd, device=dev) / Kd ** 0.5).bfloat16()
    b = torch.randn(N, device=dev)
    res = torch.randn(M, N, device=dev)
    seed = 0x1234_5678_9ABC_DEF1
    fused = K.linear(x, W, bias=b, residual=res, out_dtype=torch.float32, dropout=(0.1, seed))
    plain = K.dropout(K.linear(x, W, bias=b, out_dtype=torch.float32), 0.1, seed, res=res)[0]
    assert torch.equal(fused, plain)
    # and the torch restatement of the mask
    idx = torch.arange(M * N, device=dev, dtype=torch.int64).view(M, N)
    ref = (x.float() @ W.float().t() + b) * keep_mask(idx, seed, 0.1).float() / 0.9 + res
    assert rel(fused, ref) < 1e-4


def test_layernorm_bwd_drop(K):
    """LN backward with BERT's hidden dropout fused: the f32 output equals the plain LN backward, the
    bf16 output equals the stand-alone dropout of it, the dense-bias partials equal colsum."""
    torch.manual_seed(4)
    rows, D = 1024, 768
    x = torch.randn(rows, D, device=dev) * 2 + 0.3
    g, bt = torch.randn(D, device=dev), torch.randn(D, device=dev)
    _, _, mean, rstd = K.layernorm_fwd(x, g, bt, 1e-12)
    dy = torch.randn(rows, D, device=dev)
    seed = 0xDEAD_BEEF_0BAD_F00D
    dg1, db1, dbias1 = (torch.zeros(D, device=dev) for _ in range(3))
    dxf, dxb = K.layernorm_bwd_drop(dy, x, mean, rstd, g, 0.1, seed, dgamma_out=dg1, dbeta_out=db1, dbias_out=dbias1)
    dg0, db0 = torch.zeros(D, device=dev), torch.zeros(D, device=dev)
    ref_f, _, _, _ = K.layernorm_bwd(dy, x, mean, rstd, g, dgamma_out=dg0, dbeta_out=db0)
    ref_b = K.dropout(ref_f, 0.1, seed, out_f32=False, out_bf16=True)[1]
    torch.cuda.synchronize()
    assert torch.equal(dxf, ref_f) and torch.equal(dxb, ref_b)
    assert torch.equal(dg1, dg0) and torch.equal(db1, db0)
    assert rel(dbias1, ref_b.float().sum(0)) < 1e-5


def test_matmul_nn_gelu_bwd(K):
    """dhpre = (dy . W) * gelu'(pre) in one GEMM (act 6) vs torch fp32."""
    torch.manual_seed(5)
    M, N, Kd = 1024, 768, 3072
    dy = (torch.randn(M, N, device=dev) * 0.1).bfloat16()
    W = (torch.randn(N, Kd, device=dev) / N ** 0.5).bfloat16()
    pre = torch.randn(M, Kd, device=dev).bfloat16()
    out = K.matmul_nn_gelu_bwd(dy, W, pre)
    xp = pre.float()
    gg = 0.5 * (1 + torch.erf(xp / math.sqrt(2))) + xp * torch.exp(-0.5 * xp * xp) / math.sqrt(2 * math.pi)
    ref = (dy.float() @ W.float()) * gg
    assert rel(out.float(), ref) < 5e-3
    two = K.gelu_bwd(K.matmul_nn(dy, W), pre)
    assert rel(out.float(), two.float()) < 5e-3
