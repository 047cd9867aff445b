"""N > 1 data-parallel exchange logic on CPU (gloo, world_size 2).

The GPU path runs one process per GPU over RCCL; the exchange steps themselves
(ctclip_mi355x/dist_sync.py) are backend-agnostic host logic, exercised here with the InfoNCE
kernel replaced by the oracle's restatement (oracle.infonce, ct_clip/ct_clip.py:845-901):

  * every rank computes the same GLOBAL loss from all-gathered latents;
  * backward through each rank's own rows + one SUM all-reduce reproduces the single-process
    gradient of the global batch (encoder weights and the shared temperature);
  * summed VQ EMA statistics equal the statistics of the global batch;
  * the flat-arena trainer layout all-reduces every parameter's gradient in one collective.
"""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import ctclip_oracle as O

WORLD, B, DIN, DL = 2, 3, 16, 8


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def oracle_clip_loss(tg, ig, log_temp):
    """Same outputs as kernels.clip_loss (loss, dt, di, dlt) from the oracle's InfoNCE."""
    t = tg.detach().clone().requires_grad_(True)
    i = ig.detach().clone().requires_grad_(True)
    lt = log_temp.detach().clone().reshape(()).requires_grad_(True)
    with torch.enable_grad():          # called inside an autograd.Function forward
        tn = torch.nn.functional.normalize(t, dim=-1)
        inn = torch.nn.functional.normalize(i, dim=-1)
        loss = O.infonce(tn, inn, lt)
        loss.backward()
    return loss.detach().reshape(1), t.grad, i.grad, lt.grad.reshape(1)


def _problem():
    g = torch.Generator().manual_seed(7)
    xt = torch.randn(WORLD * B, DIN, generator=g, dtype=torch.float64).float()
    xi = torch.randn(WORLD * B, DIN, generator=g, dtype=torch.float64).float()
    wt = torch.randn(DIN, DL, generator=g, dtype=torch.float64).float()
    wi = torch.randn(DIN, DL, generator=g, dtype=torch.float64).float()
    return xt, xi, wt, wi


def _single_process():
    xt, xi, wt, wi = _problem()
    wt.requires_grad_(True)
    wi.requires_grad_(True)
    lt = torch.tensor(1.0, requires_grad=True)
    loss = O.infonce(torch.nn.functional.normalize(xt @ wt, dim=-1),
                     torch.nn.functional.normalize(xi @ wi, dim=-1), lt)
    loss.backward()
    return loss.detach(), wt.grad, wi.grad, lt.grad


def _worker(rank, port, out_dir):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=WORLD)
    try:
        from ctclip_mi355x import dist_sync
        from ctclip_mi355x.functional import ClipLossFn
        from ctclip_mi355x.trainer import FlatParams
        xt, xi, wt0, wi0 = _problem()
        wt = torch.nn.Parameter(wt0.clone())
        wi = torch.nn.Parameter(wi0.clone())
        lt = torch.nn.Parameter(torch.tensor(1.0))
        flat = FlatParams([wt, wi, lt], torch.device('cpu'))
        rows = slice(rank * B, (rank + 1) * B)
        loss = ClipLossFn.apply(xt[rows] @ wt, xi[rows] @ wi, lt, oracle_clip_loss)
        loss.backward()
        flat.rebind_grads()
        dist_sync.sum_grads(flat.grad)

        ref_loss, gwt, gwi, glt = _single_process()
        assert torch.allclose(loss.detach(), ref_loss, rtol=1e-6, atol=1e-6), (loss.item(), ref_loss.item())
        torch.testing.assert_close(wt.grad, gwt, rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(wi.grad, gwi, rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(lt.grad, glt, rtol=1e-5, atol=1e-6)
        # the arena IS the .grad storage: the single collective covered every parameter
        assert wt.grad.data_ptr() == flat.grad.data_ptr()

        # VQ EMA statistics: per-code counts and token sums of the local tokens, summed
        C, D, n = 5, 4, 7
        g = torch.Generator().manual_seed(11)
        idx = torch.randint(0, C, (WORLD, n), generator=g)
        tok = torch.randn(WORLD, n, D, generator=g)
        bins = torch.zeros(C).index_add_(0, idx[rank], torch.ones(n))
        esum = torch.zeros(C, D).index_add_(0, idx[rank], tok[rank])
        dist_sync.sum_codebook_stats(bins, esum)
        ref_bins = torch.zeros(C).index_add_(0, idx.reshape(-1), torch.ones(WORLD * n))
        ref_esum = torch.zeros(C, D).index_add_(0, idx.reshape(-1), tok.reshape(-1, D))
        assert torch.equal(bins, ref_bins)
        torch.testing.assert_close(esum, ref_esum)
        # the GPU path's 2^-40 fixed-point (int64) token sums: the cross-rank SUM is exact, so
        # every rank holds the single-process sums bit for bit
        fx = (tok * 2 ** 40).round().long()
        esum_fx = torch.zeros(C, D, dtype=torch.int64).index_add_(0, idx[rank], fx[rank])
        dist_sync.sum_codebook_stats(esum_fx)
        assert torch.equal(esum_fx, torch.zeros(C, D, dtype=torch.int64).index_add_(0, idx.reshape(-1),
                                                                                   fx.reshape(-1, D)))

        # the text latents' gather started early (CTCLIP.encode, text stream) gives the same step
        wt.grad = None
        wi.grad = None
        lt.grad = None
        t_loc = xt[rows] @ wt
        h = dist_sync.start_gather(t_loc)
        loss2 = ClipLossFn.apply(t_loc, xi[rows] @ wi, lt, oracle_clip_loss, h)
        loss2.backward()
        assert torch.equal(loss2.detach(), loss.detach())
        for prm in (wt, wi, lt):
            dist.all_reduce(prm.grad)
        torch.testing.assert_close(wt.grad, gwt, rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(lt.grad, glt, rtol=1e-5, atol=1e-6)

        # gathered latents arrive in rank order
        tg, ig = dist_sync.gather_latents(torch.full((B, DL), float(rank)), torch.full((B, DL), 10.0 + rank))
        assert torch.equal(tg[:, 0], torch.arange(WORLD).repeat_interleave(B).float())
        assert torch.equal(ig[:, 0], 10 + torch.arange(WORLD).repeat_interleave(B).float())
        open(os.path.join(out_dir, f'ok{rank}'), 'w').close()
    finally:
        dist.destroy_process_group()


def test_two_rank_contrastive_exchange(tmp_path):
    mp.spawn(_worker, args=(_free_port(), str(tmp_path)), nprocs=WORLD, join=True)
    assert all((tmp_path / f'ok{r}').exists() for r in range(WORLD))


def test_single_process_path_matches_oracle():
    """world_size 1: the same Function with no process group is the plain global loss."""
    from ctclip_mi355x.functional import ClipLossFn
    xt, xi, wt0, wi0 = _problem()
    wt = wt0.clone().requires_grad_(True)
    wi = wi0.clone().requires_grad_(True)
    lt = torch.tensor(1.0, requires_grad=True)
    loss = ClipLossFn.apply(xt @ wt, xi @ wi, lt, oracle_clip_loss)
    loss.backward()
    ref_loss, gwt, gwi, glt = _single_process()
    assert torch.allclose(loss.detach(), ref_loss)
    torch.testing.assert_close(wt.grad, gwt)
    torch.testing.assert_close(lt.grad, glt)


# ------------------------------------------------------------------ backward-overlapped buckets
class _SinkMM(torch.autograd.Function):
    """x @ w whose weight gradient is accumulated straight into w.grad inside backward, like the
    HIP layer Functions (functional.gsink)."""

    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x, w)
        return x @ w

    @staticmethod
    def backward(ctx, g):
        from ctclip_mi355x.functional import gsink
        x, w = ctx.saved_tensors
        gsink(w).add_(x.t() @ g)
        return g @ w.t(), None


class _Toy(torch.nn.Module):
    """A 3-layer text 'tower' in two readiness-ordered buckets (the top two layers, then the bottom
    one, as BertModel.grad_buckets groups layers), a 2-layer image tower and a temperature; both
    towers' backward deferred like CTCLIP's under the trainer (text first, then image)."""

    def __init__(self):
        super().__init__()
        g = torch.Generator().manual_seed(3)
        mk = lambda *s: torch.nn.Parameter(torch.randn(*s, generator=g, dtype=torch.float64).float())  # noqa: E731
        self.wt1, self.wt2, self.wt3 = mk(DIN, DIN), mk(DIN, DIN), mk(DIN, DL)
        self.wi1, self.wi2 = mk(DIN, DIN), mk(DIN, DL)
        self.lt = torch.nn.Parameter(torch.tensor(1.0))
        self.defer_text_backward = False
        self._deferred = {}

    def grad_buckets(self):
        return [('text_1', [self.wt3, self.wt2]), ('text_0', [self.wt1]), ('image', [self.wi1, self.wi2]),
                ('rest', [self.lt])]

    def _leaf(self, x, key):
        if not self.defer_text_backward:
            return x
        leaf = x.detach().requires_grad_(True)
        self._deferred[key] = (x, leaf)
        return leaf

    def backward_deferred_text(self):
        x, leaf = self._deferred.pop('text')
        torch.autograd.backward(x, leaf.grad)

    def backward_deferred_image(self):
        x, leaf = self._deferred.pop('image')
        torch.autograd.backward(x, leaf.grad)

    def forward(self, text, video, device=None, return_loss=True):
        from ctclip_mi355x import dist_sync
        from ctclip_mi355x.functional import ClipLossFn
        h = _SinkMM.apply(video, self.wi1)
        dist_sync.mark_ready(h, 'image')
        i = self._leaf(_SinkMM.apply(h, self.wi2), 'image')
        u = _SinkMM.apply(text, self.wt1)
        dist_sync.mark_ready(u, 'text_0')
        u2 = _SinkMM.apply(u, self.wt2)
        dist_sync.mark_ready(u2, 'text_1')
        t = self._leaf(_SinkMM.apply(u2, self.wt3), 'text')
        return ClipLossFn.apply(t, i, self.lt, oracle_clip_loss)


def _bucket_worker(rank, port, out_dir):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=WORLD)
    try:
        from ctclip_mi355x.trainer import CTClipTrainer
        xt, xi, _, _ = _problem()
        model = _Toy()
        ref = _Toy()
        tr = CTClipTrainer(model)
        # arena order follows the buckets, each bucket one contiguous slice
        order = ['text_1', 'text_0', 'image', 'rest']
        assert [t for t, _, _ in tr.grad_sync.buckets] == order
        assert model.wt3.grad.data_ptr() == tr.flat.grad.data_ptr()
        gs = tr.grad_sync
        fold = gs.before_launch
        rows = slice(rank * B, (rank + 1) * B)
        for step in range(2):     # hooks re-arm every step
            snaps = {}

            def snap(tag):        # the bucket's slice at the moment its all-reduce is launched
                fold(tag)
                _, off, n = next(b for b in gs.buckets if b[0] == tag)
                snaps[tag] = tr.flat.grad[off:off + n].clone()
            gs.before_launch = snap
            tr.flat.grad.zero_()
            tr.forward_backward(xt[rows], xi[rows])
            # the text buckets went out from autograd hooks during the (first-queued) text backward,
            # top layers first, then the image one; 'rest' has no hook and goes out in finish
            assert gs.launched == ['text_1', 'text_0', 'image'], gs.launched
            gs.finish()
            assert gs.launched == order
            # launched final: each bucket's local gradient at launch time is bit-identical to the
            # local gradient once the whole backward has run (sum them before the collective)
            local = {}
            for tag, off, n in gs.buckets:
                if tag in snaps:
                    local[tag] = snaps[tag]
            for tag, off, n in gs.buckets[:3]:
                assert local[tag].abs().sum().item() > 0, tag
            gs.before_launch = fold
        t = _SinkMM.apply(_SinkMM.apply(_SinkMM.apply(xt, ref.wt1), ref.wt2), ref.wt3)
        i = _SinkMM.apply(_SinkMM.apply(xi, ref.wi1), ref.wi2)
        loss = O.infonce(torch.nn.functional.normalize(t, dim=-1), torch.nn.functional.normalize(i, dim=-1), ref.lt)
        loss.backward()
        for name in ('wt1', 'wt2', 'wt3', 'wi1', 'wi2', 'lt'):
            torch.testing.assert_close(getattr(model, name).grad, getattr(ref, name).grad, rtol=1e-5, atol=1e-6)
        open(os.path.join(out_dir, f'ok{rank}'), 'w').close()
    finally:
        dist.destroy_process_group()


def test_two_rank_bucketed_overlap(tmp_path):
    """Gradient buckets all-reduced from autograd hooks during the backward (dist_sync.
    BucketedGradSync) reproduce the single-process global-batch gradient."""
    mp.spawn(_bucket_worker, args=(_free_port(), str(tmp_path)), nprocs=WORLD, join=True)
    assert all((tmp_path / f'ok{r}').exists() for r in range(WORLD))


# ------------------------------------------------------------------ eval calls issue no collective
class _StubVision(torch.nn.Module):
    def encode_pooled(self, image):
        return image, image


class _StubText(torch.nn.Module):
    def forward(self, input_ids, attention_mask=None, join=True, ready=None):
        return (input_ids[:, None, :].float(),)


def _eval_worker(rank, port, out_dir):
    """CTCLIP.forward(return_loss=False / return_encodings=True) on ONE rank must not start the
    latents' all-gather: the other rank never matches it, so the next collective
    would pair with it.  Here rank 0 scores alone, then both ranks all-reduce and compute the
    global loss; both must be exact."""
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=WORLD)
    try:
        import types
        from ctclip_mi355x import ct_clip as C
        from ctclip_mi355x import functional as Fn
        from ctclip_mi355x import kernels as K

        class _TP(torch.autograd.Function):   # f32 Linear on the CLS row (TextProjFn's math)
            @staticmethod
            def forward(ctx, cls, W):
                ctx.save_for_backward(cls, W)
                return cls @ W.t()

            @staticmethod
            def backward(ctx, g):
                cls, W = ctx.saved_tensors
                return g @ W, g.t() @ cls

        Fn.TextProjFn = _TP
        K.clip_scores = lambda t, i, lt: (torch.nn.functional.normalize(t, dim=-1)
                                          * torch.nn.functional.normalize(i, dim=-1)).sum(-1) * lt.exp()
        xt, xi, _, _ = _problem()
        torch.manual_seed(5)              # same projection weights on both ranks
        model = C.CTCLIP(image_encoder=_StubVision(), text_encoder=_StubText(), dim_text=DIN, dim_image=DIN,
                         dim_latent=DL)
        model._project = lambda W, Wb, pooled, pooled_b: pooled @ W.t()
        model._visual_weight_bf16 = lambda W: W
        rows = slice(rank * B, (rank + 1) * B)
        text = types.SimpleNamespace(input_ids=xt[rows], attention_mask=torch.ones(B, DIN))
        if rank == 0:
            with torch.no_grad():
                s = model(text, xi[rows], return_loss=False)
                enc = model(text, xi[rows], return_encodings=True)
            assert s.shape == (B,) and enc[1].shape == (B, DIN)
            assert model._t_gather is None
        probe = torch.full((4,), float(rank + 1))
        dist.all_reduce(probe)
        assert torch.equal(probe, torch.full((4,), 3.0)), probe
        # the loss path still gathers: the global InfoNCE over both ranks' pairs
        orig = Fn.ClipLossFn.apply
        C.Fn.ClipLossFn = types.SimpleNamespace(apply=lambda t, i, lt, impl, tg: orig(t, i, lt, oracle_clip_loss, tg))
        loss = model(text, xi[rows], return_loss=True)
        with torch.no_grad():
            t = torch.nn.functional.normalize(xt @ model.to_text_latent.weight.t(), dim=-1)
            i = torch.nn.functional.normalize(xi @ model.to_visual_latent.weight.t(), dim=-1)
            ref = O.infonce(t, i, model.temperature)
        assert torch.allclose(loss.detach(), ref, rtol=1e-6, atol=1e-6), (loss.item(), ref.item())
        open(os.path.join(out_dir, f'ok{rank}'), 'w').close()
    finally:
        dist.destroy_process_group()


def test_two_rank_eval_call_issues_no_collective(tmp_path):
    mp.spawn(_eval_worker, args=(_free_port(), str(tmp_path)), nprocs=WORLD, join=True)
    assert all((tmp_path / f'ok{r}').exists() for r in range(WORLD))


# ------------------------------------------------------------------ rank-consistent step skip
def _adam_ref(p, g, m, v, lr, step, skip, b1=0.9, b2=0.99, eps=1e-8):
    """torch restatement of the Adam kernel's update under its skip guard (optim.hip): a skipped
    step leaves p, m, v untouched and clears the gradient."""
    if not skip:
        m.mul_(b1).add_(g, alpha=1 - b1)
        v.mul_(b2).addcmul_(g, g, value=1 - b2)
        mh = m / (1 - b1 ** step)
        vh = v / (1 - b2 ** step)
        p.sub_(lr * mh / (vh.sqrt() + eps))
    g.zero_()


def _status_worker(rank, port, out_dir, bad_rank):
    """A LayerNorm-exchange timeout on ONE rank (its status word set) must stop the step on EVERY
    rank: the word rides the last gradient bucket's SUM all-reduce (dist_sync.BucketedGradSync
    status slot, trainer.FlatParams.status), every rank reads the same summed slot as its Adam skip
    guard and raises for the same step, and the parameter arenas stay bit-identical across ranks."""
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=WORLD)
    try:
        from ctclip_mi355x import dist_sync
        from ctclip_mi355x.trainer import FlatParams
        g = torch.Generator().manual_seed(3)
        ps = [torch.nn.Parameter(torch.randn(5, 4, generator=g)), torch.nn.Parameter(torch.randn(7, generator=g))]
        flat = FlatParams(ps, torch.device('cpu'))
        segs = [('a', 0, 20), ('b', 20, 7)]
        word = torch.zeros(1, dtype=torch.int32)
        gs = dist_sync.BucketedGradSync(flat.grad, segs, status=(flat.status, lambda: word))
        m, v = torch.zeros(flat.numel), torch.zeros(flat.numel)
        decisions = []
        for step in (1, 2, 3):
            # rank-local gradients (different on each rank), then the step's exchange
            torch.manual_seed(100 * step + rank)
            flat.grad[:flat.numel].copy_(torch.randn(flat.numel))
            if rank == bad_rank and step == 2:
                word.fill_(1)                  # this rank's fused LayerNorm exchange timed out
            gs.arm()
            gs.finish()
            skip = bool(flat.status.item() != 0)
            decisions.append(skip)
            _adam_ref(flat.data, flat.grad[:flat.numel], m, v, 1e-2, step, skip)
        # the word is sticky: steps 2 and 3 are skipped on both ranks, step 1 applied on both
        assert decisions == ([False, False, False] if bad_rank < 0 else [False, True, True]), decisions
        assert float(flat.status) == (0.0 if bad_rank < 0 else 1.0)
        both = [torch.empty_like(flat.data) for _ in range(WORLD)]
        dist.all_gather(both, flat.data)
        assert torch.equal(both[0], both[1])
        open(os.path.join(out_dir, f'ok{rank}'), 'w').close()
    finally:
        dist.destroy_process_group()


def test_two_rank_status_word_skips_every_rank(tmp_path):
    """Rank 1's LayerNorm exchange times out at step 2: both ranks skip steps 2 and 3 together."""
    mp.spawn(_status_worker, args=(_free_port(), str(tmp_path), 1), nprocs=WORLD, join=True)
    assert all((tmp_path / f'ok{r}').exists() for r in range(WORLD))


def test_two_rank_status_word_clean(tmp_path):
    """No timeout anywhere: the summed status slot stays 0 and every step is applied on both ranks."""
    mp.spawn(_status_worker, args=(_free_port(), str(tmp_path), -1), nprocs=WORLD, join=True)
    assert all((tmp_path / f'ok{r}').exists() for r in range(WORLD))


def _nan_worker(rank, port, out_dir):
    """A NaN on ONE rank (round 6 guards): at step 2 rank 1's forward flags CT_STATUS_F16_RANGE (an fp16
    copy went non-finite) and its local gradient holds a NaN.  The flag reaches every rank through the
    summed status slot; the NaN reaches every rank through the gradient SUM, so the norm the
    gradient-norm kernel takes after the all-reduce is NaN on every rank (CT_STATUS_NONFINITE_GRAD).
    Every rank skips step 2 (and, the word being sticky, step 3), raises the same NonFiniteStepError
    (trainer.raise_for_status) and keeps a parameter arena bit-identical to the other rank's."""
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=WORLD)
    try:
        from ctclip_mi355x import dist_sync
        from ctclip_mi355x.trainer import FlatParams, NonFiniteStepError, raise_for_status
        g = torch.Generator().manual_seed(5)
        ps = [torch.nn.Parameter(torch.randn(6, 3, generator=g)), torch.nn.Parameter(torch.randn(5, generator=g))]
        flat = FlatParams(ps, torch.device('cpu'))
        segs = [('a', 0, 18), ('b', 18, 5)]
        word = torch.zeros(1, dtype=torch.int32)
        gs = dist_sync.BucketedGradSync(flat.grad, segs, status=(flat.status, lambda: word))
        m, v = torch.zeros(flat.numel), torch.zeros(flat.numel)
        raised = []
        for step in (1, 2, 3):
            torch.manual_seed(100 * step + rank)
            flat.grad[:flat.numel].copy_(torch.randn(flat.numel))
            if rank == 1 and step == 2:
                word.fill_(2)                            # CT_STATUS_F16_RANGE on this rank only
                flat.grad[7] = float('nan')
            gs.arm()
            gs.finish()
            skip_word = int(flat.status.item())          # trainer: skip_word.copy_(flat.status)
            norm = flat.grad[:flat.numel].norm()
            if not torch.isfinite(norm):                 # the gradient-norm kernel's OR (optim.hip)
                skip_word |= 4
            _adam_ref(flat.data, flat.grad[:flat.numel], m, v, 1e-2, step, skip_word != 0)
            try:
                raise_for_status(skip_word, step)
                raised.append(None)
            except NonFiniteStepError as e:
                raised.append(e.bits)
        assert raised == [None, 6, 2], raised          # step 3: the sticky range bit alone
        assert torch.isfinite(flat.data).all()
        both = [torch.empty_like(flat.data) for _ in range(WORLD)]
        dist.all_gather(both, flat.data)
        assert torch.equal(both[0], both[1])
        open(os.path.join(out_dir, f'ok{rank}'), 'w').close()
    finally:
        dist.destroy_process_group()


def test_two_rank_nan_on_one_rank_skips_every_rank(tmp_path):
    mp.spawn(_nan_worker, args=(_free_port(), str(tmp_path)), nprocs=WORLD, join=True)
    assert all((tmp_path / f'ok{r}').exists() for r in range(WORLD))
