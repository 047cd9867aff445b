"""The text tower's own HIP stream.

BERT at 8 x 128 tokens is a chain of small launches (M = 1,024 rows: a few dozen workgroups
each) that leave most of the 256 CUs idle, while the 3D-ViT's launches fill the chip.  The two
towers are independent until the loss, so ``BertModel.forward`` runs on this second stream,
ordered after an event ``CTCLIP.encode`` records before it queues the image tower: the
dispatcher runs BERT's workgroups beside the ViT's.  Autograd runs every node's backward on the stream of its forward,
so BERT's backward (first in autograd order) also overlaps the ViT backward, and
its gradient bucket's all-reduce is ordered after it on this stream.  The optimizer step queues
the text bucket's Adam here too, so the next step's image tower does not wait for it (the next
BertModel.forward, on this stream, does).
``CTCLIP_TEXT_STREAM=0`` keeps everything on the current stream.

A third, auxiliary stream takes the CPB MLP (forward and, through autograd, backward: ctvit.py) and
the vector quantiser's EMA codebook update (statistics, their
all-reduce at N > 1, finalize): nothing reads the updated codebook before the next step's VQ,
which waits for it (``join_aux``)."""
from __future__ import annotations

import os

import torch

ENABLED = os.environ.get('CTCLIP_TEXT_STREAM', '1') != '0'
_STREAMS = {}


def text_stream(dev):
    """The text-tower stream of ``dev`` (None when disabled or not a GPU device)."""
    if not ENABLED or dev.type != 'cuda':
        return None
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    if idx not in _STREAMS:
        _STREAMS[idx] = torch.cuda.Stream(idx)
    return _STREAMS[idx]


def join_text(dev):
    """Order the current stream after all work queued on the text stream so far."""
    s = text_stream(dev)
    if s is not None:
        torch.cuda.current_stream(dev).wait_stream(s)


_AUX = {}
AUX_ENABLED = ENABLED and os.environ.get('CTCLIP_AUX_STREAM', '1') != '0'


def aux_stream(dev):
    """The auxiliary stream of ``dev`` (None when disabled or not a GPU device)."""
    if not AUX_ENABLED or dev.type != 'cuda':
        return None
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    if idx not in _AUX:
        _AUX[idx] = torch.cuda.Stream(idx)
    return _AUX[idx]


def join_aux(dev):
    s = aux_stream(dev)
    if s is not None:
        torch.cuda.current_stream(dev).wait_stream(s)


_MAIN = {}
# round 6 experiment: run the trainer's step on a high-priority stream (the text / aux streams keep
# the default priority), so the dispatcher prefers the critical path's workgroups when both wait
MAIN_PRIORITY = ENABLED and os.environ.get('CTCLIP_MAIN_PRIORITY', '1') != '0'


def main_stream(dev):
    """The high-priority stream the trainer's step runs on (None with CTCLIP_MAIN_PRIORITY=0)."""
    if not MAIN_PRIORITY or dev.type != 'cuda':
        return None
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    if idx not in _MAIN:
        lo, hi = torch.cuda.Stream.priority_range()
        _MAIN[idx] = torch.cuda.Stream(idx, priority=min(lo, hi))
    return _MAIN[idx]


_STATUS = {}


def status_stream(dev):
    """A stream for the trainer's per-step status-word copy to pinned host memory (None when the
    auxiliary streams are disabled): the copy is a blit kernel, and on the main stream it waited
    for CUs behind the text-bucket Adam, holding the next step's first launch back."""
    if not AUX_ENABLED or dev.type != 'cuda':
        return None
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    if idx not in _STATUS:
        _STATUS[idx] = torch.cuda.Stream(idx)
    return _STATUS[idx]


# ------------------------------------------------------------------ deferred text-stream work
# The text bucket's Adam (trainer.optimizer_step) is HBM-bound, and queued at the end of a step it
# runs beside the next step's first image-tower kernels -- the HBM-bound patch LayerNorm -- and
# slows it.  With the trainer's ``defer_text_adam`` it is handed here instead and queued by the
# next text-tower forward (``flush_text``, before BERT's own launches, so BERT still reads the
# updated weights), after an event the image tower records once its patch embedding is queued
# (``mark_image_head``): it then overlaps the image tower's later kernels instead.  ``flush_text`` is
# also the explicit flush (the trainer's ``flush``) for a step with no forward after it.
_PENDING = {}    # device index -> (fn, event recorded when fn was deferred)
_HEAD_EV = {}    # device index -> event after the image tower's patch embedding


def _idx(dev):
    return dev.index if dev.index is not None else torch.cuda.current_device()


def defer_text(dev, fn):
    """Run ``fn`` on the text stream later (see above), ordered after everything queued on the
    current stream so far."""
    if text_stream(dev) is None:
        fn()
        return
    flush_text(dev)
    _PENDING[_idx(dev)] = (fn, torch.cuda.current_stream(dev).record_event())
    _HEAD_EV.pop(_idx(dev), None)


def mark_image_head(dev, site='patch'):
    """Deferred text-stream work may start once the current stream reaches this point: the first
    call of a forward at ``MARK_SITE`` ('patch': after the patch embedding; 'attn': before the first
    spatial attention kernel, whose latency-bound launch leaves HBM idle) records the event."""
    if site != MARK_SITE or dev.type != 'cuda':
        return
    i = _idx(dev)
    if i in _PENDING and i not in _HEAD_EV:
        _HEAD_EV[i] = torch.cuda.current_stream(dev).record_event()


MARK_SITE = os.environ.get('CTCLIP_DEFER_SITE', 'attn')


def flush_text(dev):
    """Queue the deferred text-stream work now (no-op when there is none)."""
    if dev.type != 'cuda':
        return
    p = _PENDING.pop(_idx(dev), None)
    head = _HEAD_EV.pop(_idx(dev), None)
    if p is None:
        return
    fn, ev = p
    ts = text_stream(dev)
    ts.wait_event(ev)
    if head is not None:
        ts.wait_event(head)
    with torch.cuda.stream(ts):
        fn()


def pending_text(dev):
    """True while deferred text-stream work of ``dev`` waits to be queued."""
    return dev.type == 'cuda' and _idx(dev) in _PENDING


def drop_text(dev):
    """Forget the deferred work of ``dev`` (error paths)."""
    if dev.type == 'cuda':
        _PENDING.pop(_idx(dev), None)
        _HEAD_EV.pop(_idx(dev), None)
