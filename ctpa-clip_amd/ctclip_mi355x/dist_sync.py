"""Data-parallel exchange steps of the contrastive step (one process per GPU, RCCL over xGMI).

The reference runs the step under accelerate/DDP (ct_clip/CTCLIPTrainer.py:185-215, 337-340):
an all-reduce of every gradient bucket, and — through the loss — negatives drawn from the
local batch.  Here the step has exactly three exchanges, each one collective:

  1. ``gather_latents``: all-gather of the raw [B, 512] text / image latents so InfoNCE sees the
     GLOBAL batch as negatives (the text latents' gather is issued on the text stream as soon as
     BERT finishes, beside the 3D-ViT forward: ``start_gather``) (every rank then computes the same global loss; ``local_rows``
     keeps the gradient rows of this rank's pairs);
  2. ``sum_codebook_stats``: SUM of the VQ EMA statistics (per-code counts and token sums) so every
     rank applies the same codebook update (vector_quantize_pytorch's EMA with a synced codebook);
  3. ``sum_grads``: ONE SUM all-reduce over the flat f32 gradient arena (trainer.FlatParams).

Because every rank back-propagates only its own rows of a loss that is global, the SUM in (3)
reproduces the single-process gradient of the global batch exactly (tests/test_dist_gloo.py
checks this on world_size 2 with gloo).  Parameters that receive a gradient from the full
global loss on every rank (the temperature) are divided by the world size in the backward
(``replicated_grad_scale``) so the SUM counts them once.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import kernels as K
from . import streams


def world_rank():
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(), dist.get_rank()
    return 1, 0


def start_gather(x: torch.Tensor):
    """Asynchronous all-gather of this rank's [B, Dl] rows -> handle for ``finish_gather``.  RCCL
    orders it after the work already queued on the CURRENT stream only, so issuing it inside the
    producing stream's context (the text stream, streams.py) lets it run while the other stream
    keeps computing -- the side-stream latent exchange of SURVEY 8(e).  World 1: no collective."""
    world, _ = world_rank()
    x = x.detach().contiguous()
    if world == 1:
        return x, None
    B = x.shape[0]
    out = torch.empty(world * B, *x.shape[1:], device=x.device, dtype=x.dtype)
    if dist.get_backend() == 'gloo':
        work = dist.all_gather(list(out.view(world, B, *x.shape[1:]).unbind(0)), x, async_op=True)
    else:
        work = dist.all_gather_into_tensor(out, x, async_op=True)
    return out, work


def finish_gather(handle) -> torch.Tensor:
    """The gathered [world*B, Dl] tensor, with the current stream ordered after the collective."""
    out, work = handle
    if work is not None:
        work.wait()
        if out.is_cuda:
            out.record_stream(torch.cuda.current_stream(out.device))
    return out


def gather_latents(t_raw: torch.Tensor, i_raw: torch.Tensor, t_handle=None):
    """[B, Dl] x 2 on each rank -> ([world*B, Dl], [world*B, Dl]) in rank order.  ``t_handle``:
    the text latents' gather already started by ``start_gather`` (CTCLIP.encode)."""
    world, _ = world_rank()
    if world == 1:
        return t_raw.contiguous(), i_raw.contiguous()
    if t_handle is not None:
        ih = start_gather(i_raw)
        return finish_gather(t_handle), finish_gather(ih)
    B, Dl = t_raw.shape
    both = torch.cat([t_raw, i_raw], 0).contiguous()
    gathered = torch.empty(world * 2 * B, Dl, device=both.device, dtype=both.dtype)
    if dist.get_backend() == 'gloo':
        dist.all_gather(list(gathered.view(world, 2 * B, Dl).unbind(0)), both)
    else:
        dist.all_gather_into_tensor(gathered, both)
    g = gathered.view(world, 2, B, Dl)
    return g[:, 0].reshape(world * B, Dl).contiguous(), g[:, 1].reshape(world * B, Dl).contiguous()


def local_rows(x: torch.Tensor, B: int) -> torch.Tensor:
    """This rank's B rows of a [world*B, ...] global tensor."""
    _, rank = world_rank()
    return x[rank * B:(rank + 1) * B]


def replicated_grad_scale() -> float:
    world, _ = world_rank()
    return 1.0 / world


def sum_codebook_stats(*tensors: torch.Tensor) -> None:
    world, _ = world_rank()
    if world > 1:
        for t in tensors:
            dist.all_reduce(t)


def sum_grads(flat_grad: torch.Tensor) -> None:
    world, _ = world_rank()
    if world > 1:
        dist.all_reduce(flat_grad)


# ------------------------------------------------------------------ backward-overlapped buckets
# SURVEY §8(e) "Overlap": CTCLIP.encode queues the text tower first (on its own stream) and the
# image tower second, so the autograd engine (which runs the most recently created node first)
# queues the whole 3D-ViT backward before BERT's.  Each tower (or stack) marks the autograd node
# after which its parameters' .grad are final (``mark_ready``); the trainer's
# ``BucketedGradSync`` then launches that bucket's SUM all-reduce asynchronously (RCCL orders it
# after the kernels already queued on the hook's stream) while the rest of the backward keeps the
# GPU busy.  Buckets are launched in one fixed order on every rank, so the collectives match.
_READY = {}
_PENDING = {}


def mark_ready(t: torch.Tensor, tag: str) -> None:
    """Called in a forward: once ``t``'s producing node has run its backward, the parameters of
    bucket ``tag`` it owns have their final gradient.  A bucket marked on several nodes (e.g. the
    patch embedding and the CPB MLP) launches after the last of them.  No-op unless a trainer
    armed ``tag``."""
    cb = _READY.get(tag)
    if cb is None or t.grad_fn is None or not torch.is_grad_enabled():
        return
    _PENDING[tag] = _PENDING.get(tag, 0) + 1

    def fired(grad_inputs, grad_outputs):
        _PENDING[tag] -= 1
        if _PENDING[tag] == 0:
            cb(tag)
    t.grad_fn.register_hook(fired)


def disarm() -> None:
    _READY.clear()
    _PENDING.clear()


class BucketedGradSync:
    """SUM all-reduce of a flat gradient arena in contiguous buckets [(tag, offset, numel)],
    each launched as soon as its ``mark_ready`` node has run; ``finish`` launches whatever no
    hook launched (a tower without gradients, world 1) and waits for all of them."""

    def __init__(self, flat_grad: torch.Tensor, buckets, before_launch=None, force=False, status=None):
        self.grad = flat_grad
        self.buckets = list(buckets)
        # status = (slot, source): slot is the 1-element f32 view right after the last bucket in the
        # arena; just before the last bucket's all-reduce it receives source() (this rank's int32
        # status word, None = 0) and the all-reduce covers it too, so it ends up holding the SUM of
        # every rank's status -- one extra float on an existing collective, no extra launch
        self.status = status
        if status is not None and self.buckets:
            t, off, n = self.buckets[-1]
            slot = status[0]
            assert slot.data_ptr() == self.grad[off + n:off + n + 1].data_ptr(), 'status slot must follow the last bucket'
        self.before_launch = before_launch   # fold stray (non-arena) grads of a bucket
        self.force = force                   # arm the hooks even at world 1 (tests)
        self.launched = []
        self.works = []
        self.log = []
        self.stream = None

    def _launch(self, tag):
        if tag in self.launched:
            return
        # buckets go out in their fixed order: an early hook also launches every earlier bucket
        for t, off, n in self.buckets:
            if t in self.launched:
                continue
            # queued parameter-gradient reductions into this bucket (kernels.reduce_param_partials)
            # land before it is read; one queued on another stream is waited for by this one
            if K._DEFERRED:
                lo = self.grad[off:off + n].data_ptr()
                cur = torch.cuda.current_stream()
                for st in K.flush_reductions(lo, lo + 4 * n):
                    if st != cur:
                        cur.wait_stream(st)
            if self.grad.is_cuda and not t.startswith('text'):
                # an image-tower bucket may be launched from a hook on the auxiliary stream (the CPB
                # MLP's backward, ctvit.encode_tokens) or hold gradients written there: order it after
                # both the stream the step runs on and the auxiliary stream
                cur = torch.cuda.current_stream()
                if self.stream is not None and cur != self.stream:
                    cur.wait_stream(self.stream)
                streams.join_aux(self.grad.device)
            if self.before_launch is not None:
                self.before_launch(t)
            self.launched.append(t)
            self.log.append(t)
            world, _ = world_rank()
            last = self.status is not None and t == self.buckets[-1][0]
            if last:
                slot, source = self.status
                if self.grad.is_cuda and self.stream is not None:
                    # the status words are written by the forward's kernels on the step's stream
                    torch.cuda.current_stream().wait_stream(self.stream)
                src = source()
                if src is None:
                    slot.zero_()
                else:
                    slot.copy_(src)
                n += 1
            if world > 1:
                self.works.append(dist.all_reduce(self.grad[off:off + n], async_op=True))
            if t == tag:
                break

    def arm(self):
        world, _ = world_rank()
        self.launched, self.works, self.log = [], [], []
        self.stream = torch.cuda.current_stream(self.grad.device) if self.grad.is_cuda else None
        if world > 1 or self.force:
            for t, _, _ in self.buckets:
                _READY[t] = self._launch
                _PENDING[t] = 0

    def finish(self):
        for t, _, _ in self.buckets:
            _READY.pop(t, None)
            _PENDING.pop(t, None)
        if self.buckets:
            self._launch(self.buckets[-1][0])
        for w in self.works:
            w.wait()
        self.works = []
