"""Transformer building blocks with the reference's parameter layout (ct_clip/attention.py).

The modules only OWN parameters (so ``state_dict`` keys match the reference checkpoint
layout exactly); the math runs in ``functional.ViTLayerFn`` on HIP kernels.
"""
from __future__ import annotations

import torch
from torch import nn

from . import dist_sync
from . import functional as Fn


class LayerNorm(nn.Module):
    """Bias-less LayerNorm: gamma parameter, zero ``beta`` buffer (ct_clip/attention.py:28-35)."""

    def __init__(self, dim):
        super().__init__()
        self.gamma = nn.Parameter(torch.ones(dim))
        self.register_buffer('beta', torch.zeros(dim))


class GEGLU(nn.Module):
    """x, gate = chunk(2); gelu(gate) * x (ct_clip/attention.py:39-42) — fused in the FF1 GEMM."""


def FeedForward(dim, mult=4, dropout=0.):
    """Same Sequential indices as ct_clip/attention.py:44-52 (keys 0, 1, 4)."""
    inner = int(mult * (2 / 3) * dim)
    return nn.Sequential(nn.LayerNorm(dim), nn.Linear(dim, inner * 2, bias=False), GEGLU(), nn.Dropout(dropout),
                         nn.Linear(inner, dim, bias=False))


class PEG(nn.Module):
    """Causal depthwise 3x3x3 conv position generator (ct_clip/attention.py:56-84)."""

    def __init__(self, dim, causal=True):
        super().__init__()
        self.causal = causal
        self.dsconv = nn.Conv3d(dim, dim, 3, groups=dim)


class Attention(nn.Module):
    """Cosine-sim attention parameters (ct_clip/attention.py:88-125)."""

    def __init__(self, dim, dim_head=64, heads=8, num_null_kv=0, scale=8):
        super().__init__()
        self.heads = heads
        self.dim_head = dim_head
        self.scale = scale
        inner = dim_head * heads
        self.norm = LayerNorm(dim)
        self.context_norm = LayerNorm(dim)
        self.num_null_kv = num_null_kv
        self.null_kv = nn.Parameter(torch.randn(heads, 2 * num_null_kv, dim_head))
        self.to_q = nn.Linear(dim, inner, bias=False)
        self.to_kv = nn.Linear(dim, inner * 2, bias=False)
        self.q_scale = nn.Parameter(torch.ones(dim_head))
        self.k_scale = nn.Parameter(torch.ones(dim_head))
        self.to_out = nn.Linear(inner, dim, bias=False)


class ContinuousPositionBias(nn.Module):
    """CPB MLP (ct_clip/attention.py:229-276); forward returns the deduplicated table
    u[heads][(2h-1)(2w-1)] instead of the dense (heads, h*w, h*w) tensor."""

    def __init__(self, *, dim, heads, num_dims=2, layers=2):
        super().__init__()
        self.net = nn.ModuleList([nn.Sequential(nn.Linear(num_dims, dim), nn.LeakyReLU(0.1))])
        for _ in range(layers - 1):
            self.net.append(nn.Sequential(nn.Linear(dim, dim), nn.LeakyReLU(0.1)))
        self.net.append(nn.Linear(dim, heads))

    def forward(self, h, w):
        if len(self.net) != 3:
            raise NotImplementedError('CPB with layers != 2 is not on the hot path')
        rel = Fn.cpb_table(h, w, self.net[0][0].weight.device)
        return Fn.CPBFn.apply(rel, self.net[0][0].weight, self.net[0][0].bias, self.net[1][0].weight,
                              self.net[1][0].bias, self.net[2].weight, self.net[2].bias)

    def dense(self, h, w):
        """Dense (heads, h*w, h*w) bias as the reference returns it (for inspection / tests)."""
        u = self.forward(h, w)
        pos = torch.stack(torch.meshgrid(torch.arange(h), torch.arange(w), indexing='ij')).reshape(2, -1).t()
        rel = pos[:, None, :] - pos[None, :, :]
        bins = ((rel[..., 0] + h - 1) * (2 * w - 1) + (rel[..., 1] + w - 1)).to(u.device)
        return u[:, bins]


class Transformer(nn.Module):
    """Per-layer [PEG, Attention, None, FeedForward] + norm_out (ct_clip/attention.py:280-333)."""

    def __init__(self, dim, *, depth, dim_head=64, heads=8, ff_mult=4, peg=True, peg_causal=True):
        super().__init__()
        self.layers = nn.ModuleList([])
        for _ in range(depth):
            self.layers.append(nn.ModuleList([
                PEG(dim=dim, causal=peg_causal) if peg else None,
                Attention(dim=dim, dim_head=dim_head, heads=heads),
                None,
                FeedForward(dim=dim, mult=ff_mult),
            ]))
        self.norm_out = LayerNorm(dim)
        self.heads = heads
        self.dim_head = dim_head
        self.ready_tag = None   # gradient bucket tag (dist_sync.mark_ready), set by CTViT

    def run(self, xf, xb, geo, attn_bias=None):
        """x: (f32 master, bf16 shadow) rows in canonical order; returns norm_out(x) as (f32, bf16)."""
        for li, (peg, attn, _, ff) in enumerate(self.layers):
            xf, xb = Fn.ViTLayerFn.apply(
                xf, xb, attn_bias, geo, peg.dsconv.weight, peg.dsconv.bias, attn.norm.gamma, attn.q_scale,
                attn.k_scale, attn.to_q.weight, attn.to_kv.weight, attn.to_out.weight, ff[0].weight, ff[0].bias,
                ff[1].weight, ff[4].weight)
            if li == 0 and self.ready_tag:   # the stack's layer .grads are final after layer 0's backward
                dist_sync.mark_ready(xf, self.ready_tag)
        return Fn.NormFn.apply(xf, xb, self.norm_out.gamma)
