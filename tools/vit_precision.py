"""CPU experiment (oracle arithmetic): which rounding site of the bf16 3D-ViT forward drives the
pre-VQ token error (and so the VQ index flips) of the HIP path.  The model restates what the HIP
tower rounds (functional.ViTLayerFn / PatchEmbedFn), site by site:
  w     every Linear weight as bf16 (patch embed with the LayerNorm affine folded in, q | kv, out,
        FF1, FF2)
  xhat  the patch LayerNorm output (the patch-embed GEMM's A operand)
  xb    the residual stream's bf16 shadow read by the PEG conv
  x1b   the PEG output's bf16 shadow, the A operand of the Q | K | V projection
  fold  Q from rstd * (x1b (gamma o Wq)^T - mean rowsum) (the LN1 fold) instead of LN(x) Wq^T
  qkv   bf16 l2norm(q) * scale, l2norm(k) * scale, v  (qk / v: the two parts alone)
  p     the attention probabilities as bf16 (the PV MFMA operand)
  o     the attention output (to_out's A operand)
  xn2   the FeedForward LayerNorm output (FF1's A operand)
  h     FF1's output as stored (the GEGLU epilogue computes g from the rounded h, so the backward's
        recomputation matches bit for bit)
  g     the GEGLU output (FF2's A operand)
  ff1   FF1 with hi / lo split weights (w applies to FF1 only when this is off) -- "fix" probes
Each site alone and all-but-one; prints the median |l2norm(z) - l2norm(z_ref)| per token and the
VQ index flips against the f32 oracle.  Full base size, batch 1 (13,824 tokens).
  python tools/vit_precision.py [site,site,...]   (default: the standard list)"""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import ctclip_oracle as O, weights as W   # noqa: E402

torch.set_num_threads(int(os.environ.get('NT', '8')))
cfg = O.BASE.vit
P = 'visual_transformer.'
sd = {k: v for k, v in W.make_state_dict(O.BASE).items() if k.startswith(P)}
video = O.normalize_hu(W.make_hu(1, cfg))


def r(t):
    return t.bfloat16().float()


def h(t):
    return t.half().float()


def sp(t, scale=1.0):
    """split-fp16 image: hi + lo, hi = fp16(t s), lo = fp16(t s - hi) (the x3 GEMM operands)"""
    ts = t * scale
    hi = ts.half().float()
    return (hi + (ts - hi).half().float()) / scale


def rs(t, S, site):
    """site rounded as bf16 ('site'), as fp16 ('h:site'), as a split-fp16 pair ('s:site'; 'S:site'
    with the operand scaled by 2^8 first, as the x3 GEMM's weight images) or not at all"""
    if 'h:' + site in S:
        return h(t)
    if 's:' + site in S:
        return sp(t)
    if 'S:' + site in S:
        return sp(t, 256.0)
    return r(t) if site in S else t


def lin(x, w, S, site='w', name=None):
    if name is not None and any(m + 'w:' + name in S for m in ('', 'h:', 's:', 'S:')):
        return F.linear(x, rs(w, S, 'w:' + name))
    return F.linear(x, rs(w, S, site))


def patch(S):
    b, c, f, hh, ww = video.shape
    pt, ps = cfg.temporal_patch_size, cfg.patch_size
    t, h, w = f // pt, hh // ps, ww // ps
    x = video.reshape(b, c, t, pt, h, ps, w, ps).permute(0, 2, 4, 6, 1, 3, 5, 7).reshape(b, t, h, w, -1)
    g, be = sd[P + 'to_patch_emb.1.weight'], sd[P + 'to_patch_emb.1.bias']
    Wt, bt = sd[P + 'to_patch_emb.2.weight'], sd[P + 'to_patch_emb.2.bias']
    xh = rs(F.layer_norm(x, x.shape[-1:], None, None, 1e-5), S, 'xhat')
    Wf = Wt * g
    y = lin(xh, Wf, S, name='patch') + (bt + Wt @ be)
    return O._ln(y, sd[P + 'to_patch_emb.3.weight'], sd[P + 'to_patch_emb.3.bias'])


def attn(p, x1, S, bias, heads=8, dh=32):
    nb, n, d = x1.shape
    R = (lambda t, s: rs(t, S, s))
    g = sd[p + 'norm.gamma']
    Wq, Wkv = sd[p + 'to_q.weight'], sd[p + 'to_kv.weight']
    xa = R(x1, 'x1b')
    if 'fold' in S:
        Wp = g * Wq
        Wp = rs(Wp, S, 'w:q' if any(m + 'w:q' in S for m in ('', 'h:', 's:', 'S:')) else 'w')
        mean = x1.mean(-1, keepdim=True)
        rstd = torch.rsqrt(x1.var(-1, unbiased=False, keepdim=True) + 1e-5)
        q = rstd * (xa @ Wp.t() - mean * Wp.sum(1))
    else:
        q = lin(R(O._ln(x1, g, None), 'x1b'), Wq, S, name='q')
    kv = lin(xa, Wkv, S, name='kv')
    k, v = kv.chunk(2, dim=-1)

    def split(t):
        return t.reshape(nb, n, heads, dh).permute(0, 2, 1, 3)
    q, k, v = split(q), split(k), split(v)
    q = R(R(F.normalize(q, dim=-1) * sd[p + 'q_scale'], 'qkv'), 'qk')
    k = R(R(F.normalize(k, dim=-1) * sd[p + 'k_scale'], 'qkv'), 'qk')
    v = R(R(v, 'qkv'), 'v')
    sim = torch.einsum('bhid,bhjd->bhij', q, k) * 8.0
    if bias is not None:
        sim = sim + bias
    m = sim.amax(-1, keepdim=True)
    e = torch.exp(sim - m)
    den = e.sum(-1, keepdim=True)
    out = torch.einsum('bhij,bhjd->bhid', R(e, 'p'), v) / den
    out = R(out.permute(0, 2, 1, 3).reshape(nb, n, heads * dh), 'o')
    return lin(out, sd[p + 'to_out.weight'], S, name='o')


def ff(p, x2, S):
    R = (lambda t, s: rs(t, S, s))
    xn = R(O._ln(x2, sd[p + '0.weight'], sd[p + '0.bias']), 'xn2')
    W1 = sd[p + '1.weight']
    if 'ff1' in S:        # hi / lo split weights: W = bf16(W) + bf16(W - bf16(W))
        hi = r(W1)
        hh = F.linear(xn, hi + r(W1 - hi))
    else:
        h_ = lin(xn, W1, S, name='ff1')
    a, gate = R(hh if 'ff1' in S else h_, 'h').chunk(2, dim=-1)   # the GEGLU epilogue rounds h first
    gg = R(F.gelu(gate) * a, 'g')
    return lin(gg, sd[p + '4.weight'], S, name='ff2')


def stack(p, x, depth, shape, S, bias):
    for i in range(depth):
        lp = f'{p}layers.{i}.'
        x = O.peg_forward(sd, lp + '0.', rs(x, S, 'xb'), shape) + x
        x = attn(lp + '1.', x, S, bias) + x
        x = ff(lp + '3.', x, S) + x
    return O._ln(x, sd[p + 'norm_out.gamma'], sd[p + 'norm_out.beta'])


def tower(S):
    tok = patch(S)
    b, t, h, w, d = tok.shape
    shape = (b, t, h, w)
    bias = O.cpb_forward(sd, P + 'spatial_rel_pos_bias.', h, w, cfg.cpb_layers)
    x = stack(P + 'enc_spatial_transformer.', tok.reshape(b * t, h * w, d), cfg.spatial_depth, shape, S, bias)
    x = x.reshape(b, t, h, w, d).permute(0, 2, 3, 1, 4).reshape(b * h * w, t, d)
    x = stack(P + 'enc_temporal_transformer.', x, cfg.temporal_depth, shape, S, None)
    return x.reshape(b, h, w, t, d).permute(0, 3, 1, 2, 4).reshape(-1, d)


E = sd[P + 'vq._codebook.embed'][0]
with torch.no_grad():
    zr = F.normalize(tower(set()), dim=-1)
    sr = zr @ E.t()
    ir = sr.argmax(1)


def report(name, S):
    with torch.no_grad():
        z = F.normalize(tower(S), dim=-1)
        err = (z - zr).norm(dim=1)
        flips = (((z @ E.t()).argmax(1)) != ir).sum().item()
    print(f'{name:28s} |dz| median {err.median().item():.3e}  flips {flips:5d} / {ir.numel()}', flush=True)


BASE_SITES = ['w', 'xhat', 'xb', 'x1b', 'fold', 'qkv', 'p', 'o', 'xn2', 'g']
if len(sys.argv) > 1:
    for spec in sys.argv[1:]:
        report(spec, set(s for s in spec.split(',') if s))
else:
    allS = set(BASE_SITES)
    report('all (HIP default)', allS)
    for s in BASE_SITES:
        report(f'only {s}', {s})
    for s in BASE_SITES:
        report(f'all but {s}', allS - {s})
