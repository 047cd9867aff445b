"""Contrastive train step (ct_clip/CTCLIPTrainer.py:316-354) without the host data loader:
forward -> backward -> gradient all-reduce (RCCL) -> clip_grad_norm_(max_norm) -> Adam -> zero_grad.

MI355X-native layout: every trainable parameter is a view into ONE flat f32 arena, and every
.grad a view into ONE flat f32 gradient arena, so the gradient all-reduce is a single large
RCCL collective, the norm is one reduction kernel and Adam is one fused kernel (which also
never syncs the host: the clip coefficient stays on the device).
"""
from __future__ import annotations

import collections
import os

import torch


from . import dist_sync
from . import streams
from . import kernels as K

# diagnostic A/B only (CTCLIP_DIAG_TEXT_ADAM=skip | main): NOT the reference's work when 'skip'
_DIAG_TEXT_ADAM = os.environ.get('CTCLIP_DIAG_TEXT_ADAM', '')
def _ema_site():
    from . import ct_clip
    return ct_clip.DEFER_EMA


# the per-step status-word copy on its own stream (streams.status_stream); 0 = on the current stream
STATUS_COPY_STREAM = os.environ.get('CTCLIP_STATUS_COPY_STREAM', '1') != '0'


class FlatParams:
    """Every trainable parameter as a view of one f32 arena, its .grad a view of one f32 gradient
    arena, and a bf16 SHADOW arena with the same layout: the Adam kernel writes the bf16 copy of
    each updated weight as it writes the f32 one, so the forward's GEMMs read bf16 weights
    (``functional.bf``) without a cast launch per weight per step.  A shadow is trusted only while
    the parameter's torch version counter and storage are the ones recorded here (an in-place torch
    update, e.g. load_state_dict, falls back to a fresh cast until the next Adam step re-syncs)."""

    def __init__(self, params, device):
        self.params = [p for p in params if p.requires_grad]
        n = sum(p.numel() for p in self.params)
        self.numel = n
        self.data = torch.empty(n, device=device, dtype=torch.float32)
        # one element past the gradients: the step's status slot.  It rides the last gradient bucket's
        # SUM all-reduce (dist_sync.BucketedGradSync), so every rank sees the sum of the ranks'
        # LayerNorm-exchange status words and all skip (or apply) the step together.
        self.grad = torch.zeros(n + 1, device=device, dtype=torch.float32)
        self.status = self.grad[n:]
        # (shadows only on the GPU: the CPU arenas serve the gloo rehearsal tests of the sync logic)
        gpu = torch.device(device).type == 'cuda' and os.environ.get('CTCLIP_BF16_SHADOW', '1') != '0'
        self.bf16 = torch.empty(n, device=device, dtype=torch.bfloat16) if gpu else None
        # ... and its lo residual, bf16(p - bf16(p)): the text tower's GEMMs read W = hi + lo
        # (functional.bf_split, gemm.hip B2); 2 more bytes per parameter written by the same Adam pass
        self.bf16_lo = torch.empty(n, device=device, dtype=torch.bfloat16) if gpu else None
        self.views = []
        off = 0
        for p in self.params:
            k = p.numel()
            self.data[off:off + k].copy_(p.detach().reshape(-1))
            p.data = self.data[off:off + k].view_as(p)
            g = self.grad[off:off + k].view_as(p)
            p.grad = g
            if gpu:
                p._ctclip_bf16 = self.bf16[off:off + k].view_as(p)
                p._ctclip_bf16_lo = self.bf16_lo[off:off + k].view_as(p)
                p._ctclip_off = off
                p._ctclip_flat = self
            self.views.append((off, k, g))
            off += k
        if gpu and n:
            K.cast_bf16_split(self.data, hi=self.bf16, lo=self.bf16_lo)
            self.sync_shadows(0, n)

    def sync_shadows(self, lo, hi):
        """Mark the shadows of the parameters in [lo, hi) current (after the kernel that wrote them)."""
        if self.bf16 is None:
            return
        for p, (off, k, _) in zip(self.params, self.views):
            if lo <= off < hi:
                p._ctclip_ver = p._version
                p._ctclip_ptr = p.data_ptr()

    def rebind_grads(self, only=None):
        """Make sure every .grad is (still) the arena view; fold stray grads back in."""
        sel = None if only is None else {id(p) for p in only}
        for p, (off, k, g) in zip(self.params, self.views):
            if sel is not None and id(p) not in sel:
                continue
            if p.grad is None:
                p.grad = g
            elif p.grad.data_ptr() != g.data_ptr():
                g.copy_(p.grad)
                p.grad = g


class StepGuardError(RuntimeError):
    """A training step was flagged on the device and NOT applied: the summed step status words
    (include/ctclip_hip.h CT_STATUS_*) are the Adam kernels' skip guard, so no rank changed its
    parameters or moments (the gradients were cleared), and the codebook EMA of that step was dropped.
    ``bits`` holds the (rank-summed) status value.  The status word is sticky: later steps are skipped
    too until ``kernels.reset_ln_status()``."""

    def __init__(self, msg, bits=0):
        super().__init__(msg)
        self.bits = bits


class LayerNormExchangeError(StepGuardError):
    """A LayerNorm-fused GEMM (kernels.linear_residual_ln, gemm256.hip EP -6 / -7) gave up waiting for
    its partner tile's row statistics: that step's LayerNorm outputs were wrong.  The step's Adam
    update was not applied (the status word is the Adam kernel's skip guard); later steps are not
    applied either until ``kernels.reset_ln_status()``."""


class NonFiniteStepError(StepGuardError):
    """The step's forward or gradients left the representable range: an fp16 operand copy saturated or
    was non-finite (CT_STATUS_F16_RANGE, the 16-bit image-tower forward), a token reached the vector
    quantiser without a finite score (CT_STATUS_VQ_NONFINITE), or the gradient norm was NaN / inf
    (CT_STATUS_NONFINITE_GRAD).  The reference's fp32 step would have propagated the NaN into every
    parameter; here no rank applied the step."""


_STATUS_NAMES = ((1, 'LayerNorm exchange timeout'), (2, 'fp16 range (saturated / non-finite fp16 operand)'),
                 (4, 'non-finite gradient norm'), (8, 'non-finite VQ token'))


def describe_status(v):
    """Names of the status bits of a (single-rank) status value."""
    return ', '.join(n for b, n in _STATUS_NAMES if v & b) or 'none'


def raise_for_status(v, step):
    """Raise the StepGuardError of a step's skip word ``v`` (the ranks' summed status words, with the
    gradient-norm bit ORed in), if it is nonzero.  Every rank holds the same value, so every rank
    raises for the same step."""
    if v == 0:
        return
    if v == 1:
        raise LayerNormExchangeError(
            f'LayerNorm-fused GEMM exchange timed out (status word set by step {step} or earlier, on '
            'this rank or another: the ranks\' words are summed with the gradients): its LayerNorm '
            'outputs were wrong and the Adam update of that step was skipped on every rank; '
            'kernels.reset_ln_status() clears the word (CTCLIP_LN_FUSED=0 runs the unfused GEMM + '
            'LayerNorm pair instead)', bits=v)
    raise NonFiniteStepError(
        f'step {step} (or earlier) was flagged on the device, status {v} ({describe_status(v)}; summed '
        'over the ranks): its Adam update and codebook EMA were skipped on every rank, parameters and '
        'moments unchanged; kernels.reset_ln_status() clears the sticky word', bits=v)


# queue BERT's backward before the 3D-ViT's (CTCLIP_TEXT_FIRST=0: after it, the r02 order; A/B)
TEXT_FIRST = os.environ.get('CTCLIP_TEXT_FIRST', '1') != '0'


def grad_buckets(model):
    """[(tag, params)] with every parameter in exactly one bucket, in the model's readiness order
    (``model.grad_buckets()``, e.g. CTCLIP: BERT layer groups, vit_temporal, vit_spatial, vit_rest,
    head)."""
    if not hasattr(model, 'grad_buckets'):
        spec = [('all', list(model.parameters()))]
    else:
        try:
            spec = model.grad_buckets(text_first=TEXT_FIRST)
        except TypeError:
            spec = model.grad_buckets()
    seen, out = set(), []
    for tag, ps in spec:
        mine = []
        for p in ps:
            if id(p) not in seen:
                seen.add(id(p))
                mine.append(p)
        out.append((tag, mine))
    rest = [p for p in model.parameters() if id(p) not in seen]
    if rest:
        out[-1][1].extend(rest)
    return out


class CTClipTrainer:
    """Optimiser + step for a ``ctclip_mi355x.CTCLIP``.  Hyper-parameters default to the
    reference's (CTCLIPTrainer.py:203-205, optimizer.py:24: Adam lr 1.25e-6, betas (0.9, 0.99),
    eps 1e-8, wd 0, clip 0.5)."""

    def __init__(self, model, lr=1.25e-6, wd=0.0, max_grad_norm=0.5, betas=(0.9, 0.99), eps=1e-8,
                 overlap_grad_sync=True, defer_text_adam=False):
        self.model = model
        # the text bucket's Adam is queued by the NEXT step's text-tower forward (streams.defer_text);
        # call flush() after the last train_step before reading the parameters
        self.defer_text_adam = defer_text_adam
        dev = next(model.parameters()).device
        self.device = dev
        # arena order = gradient bucket order, so every bucket is one contiguous slice
        groups = grad_buckets(model) if overlap_grad_sync else [('all', list(model.parameters()))]
        self.flat = FlatParams([p for _, ps in groups for p in ps], dev)
        segs, off, self.bucket_params = [], 0, {}
        for tag, ps in groups:
            n = sum(p.numel() for p in ps if p.requires_grad)
            if n:
                segs.append((tag, off, n))
                self.bucket_params[tag] = [p for p in ps if p.requires_grad]
            off += n
        self.grad_sync = dist_sync.BucketedGradSync(self.flat.grad, segs, before_launch=self._fold_bucket,
                                                    status=(self.flat.status, self._local_status))
        self.m = torch.zeros_like(self.flat.data)
        self.v = torch.zeros_like(self.flat.data)
        self.lr, self.wd, self.max_grad_norm, self.betas, self.eps = lr, wd, max_grad_norm, betas, eps
        self.steps = 0
        self.norm = torch.zeros(2, device=dev, dtype=torch.float32)
        # the Adam kernels' skip guard of step s: skip_ring[s % 4] = (summed status slot != 0), written
        # after the all-reduce; a ring so a deferred text-bucket Adam still reads its own step's word
        self.skip_ring = torch.zeros(4, device=dev, dtype=torch.int32)
        self.world = dist_sync.world_rank()[0]
        # per-step host check of the LayerNorm-fused GEMMs' status word (kernels.ln_guard): an async
        # copy into pinned memory after each step, read once its event completed -- never more than
        # two steps after the step it covers, so the host stays up to two steps ahead of the GPU
        self._guard = dev.type == 'cuda'
        self._ln_pending = collections.deque()       # (step, event, pinned int32[1])
        self._ln_host = [torch.zeros(1, dtype=torch.int32, pin_memory=True) for _ in range(4)] if self._guard else []
        self.ln_steps_checked = 0

    def _local_status(self):
        """This rank's sticky LayerNorm-exchange status word (int32[1] on the device), or None (CPU)."""
        return K.ln_status_tensor(self.device) if self._guard else None

    def _fold_bucket(self, tag):
        self.flat.rebind_grads(self.bucket_params.get(tag, ()))

    def forward_backward(self, text, video):
        self.grad_sync.arm()
        defer = hasattr(self.model, 'backward_deferred_text')
        if defer:
            self.model.defer_text_backward = True
        try:
            loss = self.model(text, video, device=self.device, return_loss=True)
            loss.backward()                      # the loss node (both towers' latents are leaves)
            if defer:
                # BERT first (text stream): its layer-group buckets go out to RCCL as its backward
                # finalises them, ahead of the 3D-ViT's (main stream), whose backward runs beside it
                # (TEXT_FIRST = False: the r02 order, 3D-ViT queued first)
                back_img = getattr(self.model, 'backward_deferred_image', None)
                if not TEXT_FIRST and back_img is not None:
                    back_img()
                self.model.backward_deferred_text()
                if TEXT_FIRST and back_img is not None:
                    back_img()
        except BaseException:
            dist_sync.disarm()
            K.discard_deferred()
            raise
        finally:
            if defer:
                self.model.defer_text_backward = False
        return loss

    def optimizer_step(self):
        try:
            self._optimizer_step()
        finally:
            vqs = getattr(self.model, '_vq_state', lambda: None)()
            if vqs is not None and vqs.pending_ema is not None and self._guard:
                # the pending update is guarded by this step's summed skip word (forward flags of
                # every rank + a non-finite gradient norm), whenever it runs
                vqs.ema_guard = self.skip_ring[self.steps % 4:self.steps % 4 + 1]
            fe = getattr(self.model, 'flush_ema', None)
            if fe is not None and _ema_site() != '3':
                fe()      # a codebook EMA train_step deferred past the optimizer (ct_clip.DEFER_EMA '2';
                #           '3': the next step's image tower queues it after its patch embedding)

    def _optimizer_step(self):
        if streams.pending_text(self.device):
            # the previous step's deferred text Adam was never queued (no text-tower forward ran
            # since): this step's text gradients were summed onto that step's and the shared clip
            # coefficient is about to be overwritten -- refuse rather than train on mixed gradients
            streams.drop_text(self.device)
            raise RuntimeError('CTClipTrainer: a deferred text-tower Adam is still pending at optimizer_step '
                               '(defer_text_adam needs a text-tower forward between optimizer steps; call '
                               'flush() after the last train_step)')
        # SUM (ClipLossFn gives each rank its own rows): buckets already in flight since their
        # tower's backward finished; the last one goes out here and all are waited on.  BERT's
        # backward ran on the text stream (streams.py): order the norm / Adam after it.
        streams.join_text(self.device)
        streams.join_aux(self.device)     # the VQ EMA update (already done by now; keeps state coherent)
        self.grad_sync.finish()
        self.steps += 1
        skip_word = self.skip_ring[self.steps % 4:self.steps % 4 + 1]
        # the ranks' summed status words (any rank flagged -> all skip); the norm kernel ORs in a
        # non-finite gradient (the norm of the all-reduced gradient: the same on every rank)
        skip_word.copy_(self.flat.status)
        K.grad_norm(self.flat.grad[:self.flat.numel], self.max_grad_norm if self.max_grad_norm else 0.0, self.norm,
                    skip=skip_word if self._guard else None)
        # the text bucket's Adam (and grad reset) goes on the text stream: the next step's image
        # tower does not wait for it, the next step's BERT (same stream) does.  It is queued
        # behind the 3D-ViT's Adam (main stream), not beside it: both are HBM-bound, and run side
        # by side the small 3D-ViT update (~25 M parameters) finished only with the large BERT one
        # (~110 M), holding the next step's image tower back by ~0.8 ms; queued after it, the
        # BERT update overlaps the next step's compute-bound image-tower GEMMs instead.
        ts = streams.text_stream(self.device)
        text = [b for b in self.grad_sync.buckets if b[0].startswith('text')] if ts is not None else []
        skip = []
        if text:          # the text buckets are adjacent in the arena (one slice)
            off = min(b[1] for b in text)
            n = sum(b[2] for b in text)
            assert max(b[1] + b[2] for b in text) == off + n
            skip = [(off, n)]
        lo = 0
        for off, n in skip + [(self.flat.numel, 0)]:
            if off > lo:
                self._adam(lo, off - lo)
            lo = off + n
        if skip and _DIAG_TEXT_ADAM == 'skip':     # diagnostic only: what the overlap costs
            return
        if skip and _DIAG_TEXT_ADAM == 'main':     # diagnostic only: serialised on the main stream
            off, n = skip[0]
            self._adam(off, n)
            return
        if skip and self.defer_text_adam:
            # queued by the next step's BERT forward, after the next image tower's patch embedding
            # (streams.defer_text); ``flush`` queues it when no step follows
            off, n = skip[0]
            step = self.steps
            streams.defer_text(self.device, lambda: self._adam(off, n, step=step))
            return
        if skip:
            off, n = skip[0]
            ts.wait_stream(torch.cuda.current_stream(self.device))   # clip coefficient ready
            with torch.cuda.stream(ts):
                self._adam(off, n)

    def flush(self):
        """Queue any deferred text-bucket Adam (``defer_text_adam``) now and verify every step's
        LayerNorm-exchange status (synchronises): call after the last ``train_step`` before reading
        the parameters."""
        streams.flush_text(self.device)
        fe = getattr(self.model, 'flush_ema', None)
        if fe is not None:
            fe()
        # the text-bucket Adam runs on the text stream, the codebook EMA on the auxiliary one: order
        # the caller's stream after both, so parameters read (or saved) on it are the updated ones
        streams.join_text(self.device)
        streams.join_aux(self.device)
        self.check()

    def check(self):
        """Wait for every queued step-status copy and raise LayerNormExchangeError if a step's
        LayerNorm-fused GEMM timed out."""
        self._check_ln(block_upto=self.steps)

    def _queue_ln_check(self):
        if not self._guard:
            return
        host = self._ln_host[self.steps % len(self._ln_host)]
        # the step's skip word (the ranks' summed status): every rank raises for the same step.  The
        # copy goes on its own stream (STATUS_COPY_STREAM), ordered after the current stream's work so
        # far: the next step's first launches do not queue behind its blit kernel
        cs = streams.status_stream(self.device) if STATUS_COPY_STREAM else None
        ev = torch.cuda.Event()
        if cs is not None:
            cs.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(cs):
                host.copy_(self.skip_ring[self.steps % 4:self.steps % 4 + 1], non_blocking=True)
                ev.record()
        else:
            host.copy_(self.skip_ring[self.steps % 4:self.steps % 4 + 1], non_blocking=True)
            ev.record()
        self._ln_pending.append((self.steps, ev, host))

    def _check_ln(self, block_upto):
        """Consume the status copies: those of steps <= block_upto are waited for, newer ones are
        read only if already complete."""
        while self._ln_pending:
            step, ev, host = self._ln_pending[0]
            if step <= block_upto:
                ev.synchronize()
            elif not ev.query():
                break
            self._ln_pending.popleft()
            v = int(host[0])
            if v != 0:
                self._ln_pending.clear()
                raise_for_status(v, step)
            self.ln_steps_checked = step

    def _adam(self, off, n, step=None):
        sl = slice(off, off + n)
        st = self.steps if step is None else step
        K.adam(self.flat.data[sl], self.flat.grad[sl], self.m[sl], self.v[sl], lr=self.lr, b1=self.betas[0],
               b2=self.betas[1], eps=self.eps, wd=self.wd, step=self.steps if step is None else step, coef=self.norm,
               p_bf16=self.flat.bf16[sl] if self.flat.bf16 is not None else None,
               p_bf16_lo=self.flat.bf16_lo[sl] if self.flat.bf16_lo is not None else None, zero_grad=True,
               skip=self.skip_ring[st % 4:st % 4 + 1] if self._guard else None)
        self.flat.sync_shadows(off, off + n)

    def train_step(self, text, video):
        """One contrastive step; returns the loss tensor (no host sync).  Raises
        LayerNormExchangeError once the status copy of an earlier step shows a timed-out LayerNorm
        exchange (at the latest two steps later; ``check()`` / ``flush()`` wait for all)."""
        hp = streams.main_stream(self.device)
        if hp is None:
            return self._train_step(text, video)
        # CTCLIP_MAIN_PRIORITY=1: the step on the high-priority stream, ordered after the caller's
        # work so far, and the caller's stream after it
        caller = torch.cuda.current_stream(self.device)
        hp.wait_stream(caller)
        with torch.cuda.stream(hp):
            loss = self._train_step(text, video)
        caller.wait_stream(hp)
        loss.record_stream(caller)
        return loss

    def _train_step(self, text, video):
        self._check_ln(block_upto=self.steps - 2)
        self.model.train()
        own = hasattr(self.model, 'ema_after_step')
        if own:
            self.model.ema_after_step = True     # the codebook EMA goes after optimizer_step
        try:
            with K.ln_guard():
                loss = self.forward_backward(text, video)
        finally:
            if own:
                self.model.ema_after_step = False
        self.optimizer_step()
        self._queue_ln_check()
        return loss.detach()
