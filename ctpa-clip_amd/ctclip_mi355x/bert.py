"""BERT-base text encoder on HIP kernels with ``transformers.BertModel``'s state_dict layout
(the reference's text tower, ct_clip/pretrained_model.py:9, called at ct_clip/ct_clip.py:685-686).

``forward(input_ids, attention_mask)`` returns a tuple whose [0] is last_hidden_state, like
the HF model output indexed by the reference (``text_embeddings[0]``).  In train mode HF's
dropout (p = 0.1) is applied at its four sites -- embeddings, attention probabilities (inside
the fused attention kernels), attention output and FF output -- with hash masks regenerated in
the backward.  The pooler's parameters are kept for checkpoint
compatibility; the pooler output is unused by CT-CLIP and is not computed.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch
from torch import nn

from . import dist_sync
from . import functional as Fn
from . import streams


# diagnostic only (A/B of what the dropout sites cost): CTCLIP_BERT_NODROP=1 runs train mode without
# dropout, which is NOT the reference's work
_NO_DROP = os.environ.get('CTCLIP_BERT_NODROP', '0') != '0'


@dataclass
class BertConfig:
    vocab_size: int = 30522
    hidden_size: int = 768
    num_hidden_layers: int = 12
    num_attention_heads: int = 12
    intermediate_size: int = 3072
    max_position_embeddings: int = 512
    type_vocab_size: int = 2
    layer_norm_eps: float = 1e-12
    hidden_dropout_prob: float = 0.1
    attention_probs_dropout_prob: float = 0.1
    pad_token_id: int = 0


class _Embeddings(nn.Module):
    def __init__(self, c):
        super().__init__()
        # padding_idx as transformers' BertEmbeddings: the pad row gets no gradient
        self.word_embeddings = nn.Embedding(c.vocab_size, c.hidden_size, padding_idx=c.pad_token_id)
        self.position_embeddings = nn.Embedding(c.max_position_embeddings, c.hidden_size)
        self.token_type_embeddings = nn.Embedding(c.type_vocab_size, c.hidden_size)
        self.LayerNorm = nn.LayerNorm(c.hidden_size, eps=c.layer_norm_eps)


class _SelfAttn(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.query = nn.Linear(c.hidden_size, c.hidden_size)
        self.key = nn.Linear(c.hidden_size, c.hidden_size)
        self.value = nn.Linear(c.hidden_size, c.hidden_size)


class _DenseLN(nn.Module):
    def __init__(self, din, dout, eps):
        super().__init__()
        self.dense = nn.Linear(din, dout)
        self.LayerNorm = nn.LayerNorm(dout, eps=eps)


class _Attention(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.self = _SelfAttn(c)
        self.output = _DenseLN(c.hidden_size, c.hidden_size, c.layer_norm_eps)


class _Dense(nn.Module):
    def __init__(self, din, dout):
        super().__init__()
        self.dense = nn.Linear(din, dout)


class BertLayer(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.attention = _Attention(c)
        self.intermediate = _Dense(c.hidden_size, c.intermediate_size)
        self.output = _DenseLN(c.intermediate_size, c.hidden_size, c.layer_norm_eps)


class _Encoder(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.layer = nn.ModuleList([BertLayer(c) for _ in range(c.num_hidden_layers)])


class BertModel(nn.Module):
    def __init__(self, config: BertConfig = None, **kw):
        super().__init__()
        self.config = config or BertConfig(**kw)
        c = self.config
        if (c.hidden_size // c.num_attention_heads) not in (32, 64):
            raise NotImplementedError('HIP attention kernels support head dim 32 or 64')
        self.embeddings = _Embeddings(c)
        self.encoder = _Encoder(c)
        self.pooler = _Dense(c.hidden_size, c.hidden_size)
        for m in self.modules():   # BERT init (std 0.02)
            if isinstance(m, (nn.Linear, nn.Embedding)):
                nn.init.normal_(m.weight, std=0.02)
            if isinstance(m, nn.Linear):
                nn.init.zeros_(m.bias)

    bucket_layers = 3     # encoder layers per gradient all-reduce bucket (grad_buckets)

    def _layer_params(self, li):
        lyr = self.encoder.layer[li]
        a = lyr.attention.self
        first = [a.query.weight, a.key.weight, a.value.weight, a.query.bias, a.key.bias, a.value.bias]
        ids = {id(p) for p in first}
        return first + [p for p in lyr.parameters() if id(p) not in ids]

    def _bucket_groups(self):
        """[(lo, hi)] layer ranges, top of the stack first (the order the backward finalises them)."""
        n, k = len(self.encoder.layer), max(1, int(self.bucket_layers))
        out, hi = [], n
        while hi > 0:
            out.append((max(0, hi - k), hi))
            hi = max(0, hi - k)
        return out

    def grad_buckets(self):
        """[(tag, params)] in the order BERT's backward finalises them, like DDP's readiness-ordered
        buckets (ct_clip/CTCLIPTrainer.py:213-217): every ``bucket_layers`` encoder layers from the
        top down, the lowest group together with the embeddings (and the unused pooler).  Each
        layer's query / key / value weights then biases stay adjacent, so the fused QKV GEMM reads
        them as one slice of the trainer's arenas (functional.bf_cat).  The forward marks each
        group's lowest layer (dist_sync.mark_ready) so its all-reduce goes out as soon as that
        layer's backward has run -- beside the rest of BERT's backward and the 3D-ViT's."""
        groups = self._bucket_groups()
        out = []
        for lo, hi in groups:
            ps = []
            for li in range(hi - 1, lo - 1, -1):
                ps += self._layer_params(li)
            out.append((f'text_{lo}', ps))
        seen = {id(p) for _, ps in out for p in ps}
        out[-1][1].extend(p for p in self.parameters() if id(p) not in seen)
        return out

    def param_order(self):
        """All parameters, each layer's query / key / value weights then biases first and adjacent,
        so the fused QKV GEMM reads them as one slice of the trainer's arenas (functional.bf_cat)."""
        first = []
        for lyr in self.encoder.layer:
            a = lyr.attention.self
            first += [a.query.weight, a.key.weight, a.value.weight, a.query.bias, a.key.bias, a.value.bias]
        ids = {id(p) for p in first}
        return first + [p for p in self.parameters() if id(p) not in ids]

    def forward(self, input_ids, attention_mask=None, join=True, ready=None, **_):
        """Runs on the text stream (streams.py) when there is one, ordered after ``ready`` (an event
        of the calling stream; default: everything queued on it so far) and after the previous
        optimizer step's Adam of these weights (queued on the text stream).  ``join``: the calling
        stream waits for the result before this returns; with join=False the caller joins later
        (``streams.join_text``).  Backward nodes run on the text stream."""
        dev = input_ids.device
        ts = streams.text_stream(dev)
        if ts is None:
            return self._forward(input_ids, attention_mask)
        cur = torch.cuda.current_stream(dev)
        streams.flush_text(dev)        # a deferred Adam of these weights (trainer.defer_text_adam)
        if ready is not None:
            ts.wait_event(ready)
        else:
            ts.wait_stream(cur)
        for t in (input_ids, attention_mask):
            if t is not None and t.is_cuda:
                t.record_stream(ts)
        with torch.cuda.stream(ts):
            out = self._forward(input_ids, attention_mask)
        out[0].record_stream(cur)
        if join:
            cur.wait_stream(ts)
        return out

    def _forward(self, input_ids, attention_mask=None):
        c = self.config
        B, L = input_ids.shape
        ids = input_ids.to(torch.int64).contiguous()
        if attention_mask is None:
            attention_mask = torch.ones_like(ids)
        kmask = attention_mask.to(torch.int32).contiguous()
        e = self.embeddings
        # train-mode dropout (HF BertEmbeddings / BertSelfAttention / BertSelfOutput / BertOutput):
        # one 64-bit seed per (forward call, layer, site); the masks are hashes of it (no host RNG state
        # on the step path, the backward regenerates them)
        ph = float(c.hidden_dropout_prob) if self.training and not _NO_DROP else 0.0
        pa = float(c.attention_probs_dropout_prob) if self.training and not _NO_DROP else 0.0
        self._drop_calls = getattr(self, '_drop_calls', 0) + 1
        base = (torch.initial_seed() * 0x2545F4914F6CDD1D + self._drop_calls * 0x9E3779B97F4A7C15) & (2 ** 64 - 1)

        def seed(layer, site):
            return (base ^ ((layer * 4 + site + 1) * 0xBF58476D1CE4E5B9)) & (2 ** 64 - 1)

        xf, xb = Fn.BertEmbedFn.apply(ids, e.word_embeddings.weight, e.position_embeddings.weight,
                                      e.token_type_embeddings.weight, e.LayerNorm.weight, e.LayerNorm.bias,
                                      c.layer_norm_eps, (ph, seed(0, 3)), c.pad_token_id)
        # gradient buckets (grad_buckets): the lowest group's .grad are final once the embeddings'
        # backward ran, every other group's once its lowest layer's backward ran
        lows = {lo for lo, _ in self._bucket_groups()}
        dist_sync.mark_ready(xf, 'text_0')
        for li, lyr in enumerate(self.encoder.layer):
            a = lyr.attention
            xf, xb = Fn.BertLayerFn.apply(
                xf, xb, kmask, B, L, c.num_attention_heads, c.layer_norm_eps,
                a.self.query.weight, a.self.query.bias, a.self.key.weight, a.self.key.bias,
                a.self.value.weight, a.self.value.bias, a.output.dense.weight, a.output.dense.bias,
                a.output.LayerNorm.weight, a.output.LayerNorm.bias, lyr.intermediate.dense.weight,
                lyr.intermediate.dense.bias, lyr.output.dense.weight, lyr.output.dense.bias,
                lyr.output.LayerNorm.weight, lyr.output.LayerNorm.bias,
                (ph, pa, seed(li + 1, 0), seed(li + 1, 1), seed(li + 1, 2)),
                li >= len(self.encoder.layer) - Fn._TEXT_SPLIT_LAYERS)
            if li in lows and li > 0:
                dist_sync.mark_ready(xf, f'text_{li}')
        return (xf.view(B, L, c.hidden_size), None)
