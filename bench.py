"""Benchmark: CT-CLIP contrastive train step on MI355X (BASELINE.json metric: CT-report pairs/s).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
    (N > 1: one rank per GPU over RCCL -- under torch.distributed.run, or, when started without a
    launcher, bench.py starts torch.distributed.run --nproc-per-node N itself as a child process)

A step = CTCLIP forward (BERT-base text tower on 128-token reports + CTViT base image tower on
int16-HU 240x480x480 volumes + projections + InfoNCE over the all-gathered global batch) ->
backward -> RCCL gradient all-reduce -> clip_grad_norm_(0.5) -> Adam, with every weight trained
that the reference fine-tunes (ct_clip/fine_tuning_ctclip.py:6-14).  Inputs are synthetic and
generated on the device before the timed region; weights are random-init of the same
architecture (no network for checkpoints).  Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
import types

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, 'ctpa-clip_amd'))
sys.path.insert(0, REPO)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

PEAK_BF16_TFLOPS = 2500.0     # MI355X dense bf16 MFMA (MI355X_MICROARCH.md, chip-level parameters)
PEAK_HBM_GBS = 8000.0
VIT_FWD_GFLOP_PER_VOL = 789.33 + 1.18   # 3D-ViT forward + deduplicated CPB


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--batch', type=int, default=None,
                    help='volume/report pairs per GPU (configs[1]: 8; configs[3] with --fp8: 16)')
    ap.add_argument('--fp8', action='store_true',
                    help='configs[3]: the 3D-ViT forward linears as MX-fp8 GEMMs (default batch 16 per GPU)')
    ap.add_argument('--text-len', type=int, default=128)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--f32-tower', action='store_true',
                    help="run the whole bench in the f32 image-tower mode (= --vit-precision f32)")
    ap.add_argument('--vit-precision', default=None, choices=['bf16', 'f32', 'split'],
                    help='run the whole bench in this image-tower mode (precise.set_vit_precision; profiling)')
    ap.add_argument('--no-eval-forward', action='store_true',
                    help='skip the eval-mode forward measurement (vit_forward_eval; e.g. under a profiler)')
    ap.add_argument('--no-precise', action='store_true',
                    help='skip the precise image-tower measurements (precise_split_tower / precise_f32_tower)')
    ap.add_argument('--cpu-batch', type=int, default=2)
    ap.add_argument('--dist-backend', default='nccl', choices=['nccl', 'gloo'],
                    help='gloo: rehearse the N>1 path with several ranks sharing one GPU (not a bench number)')
    return ap.parse_args()


def synthetic_inputs(B, L, rank, device, frames=240, size=480, vocab=30522):
    g = torch.Generator(device=device)
    g.manual_seed(1234 + rank)
    hu = torch.randint(-1200, 1201, (B, 1, frames, size, size), generator=g, device=device,
                       dtype=torch.int32).to(torch.int16)
    g.manual_seed(4321 + rank)
    ids = torch.randint(5, vocab, (B, L), generator=g, device=device)
    ids[:, 0] = 2
    ids[:, -1] = 3
    mask = torch.ones(B, L, dtype=torch.long, device=device)
    return hu, types.SimpleNamespace(input_ids=ids, attention_mask=mask)


def cpu_baseline(batch, runs=3):
    """The oracle (fp32 eager CPU restatement of the reference, pinned by tests/golden) timed on
    this host, per SURVEY 8(d) / BASELINE.md: one full contrastive step (fwd + bwd + clip + Adam) at
    batch `batch`, base config, all host threads; one untimed warm-up step, then the MEDIAN of
    `runs` timed steps."""
    import statistics
    from oracle import ctclip_oracle as O
    from oracle import weights as W
    # BASELINE.md / SURVEY 8(d) ask for torch.set_num_threads(os.cpu_count()).  On the GPU box
    # os.cpu_count() reports the whole host (all logical CPUs) while this process's cgroup gets a
    # share of them (16 for one GPU, also exported as OMP_NUM_THREADS): more threads than that share
    # only time-slice.  So: os.cpu_count(), capped by the cgroup CPU quota and OMP_NUM_THREADS,
    # each cap stated in the line.
    threads = os.cpu_count() or 1
    caps = []
    quota = _cgroup_cpus()
    if quota is not None and quota < threads:
        threads = quota
        caps.append(f'cgroup CPU quota {quota}')
    omp = os.environ.get('OMP_NUM_THREADS')
    if omp and omp.isdigit() and int(omp) < threads:
        threads = int(omp)
        caps.append(f'OMP_NUM_THREADS={omp}')
    torch.set_num_threads(threads)
    cfg = O.BASE
    sd = W.make_state_dict(cfg)
    params = []
    for k, v in sd.items():
        if k.startswith(O.trainable_prefixes()) and v.is_floating_point() and 'vq._codebook' not in k \
                and not k.endswith('beta') and v.numel():
            v.requires_grad_(True)
            params.append(v)
    opt = torch.optim.Adam(params, lr=1.25e-6, betas=(0.9, 0.99), eps=1e-8)
    ids, mask = W.make_text(batch, 128, cfg.bert.vocab_size)
    video = O.normalize_hu(W.make_hu(batch, cfg.vit))

    def step():
        t0 = time.perf_counter()
        out = O.ctclip_forward(sd, ids, mask, video, cfg, training=True)
        out['loss'].backward()
        torch.nn.utils.clip_grad_norm_(params, 0.5)
        opt.step()
        opt.zero_grad()
        return time.perf_counter() - t0

    warm = step()
    print(f'cpu_baseline: warm-up step {warm:.1f} s', file=sys.stderr, flush=True)
    times = []
    for i in range(runs):
        times.append(step())
        print(f'cpu_baseline: step {i + 1}/{runs} {times[-1]:.1f} s', file=sys.stderr, flush=True)
    dt = statistics.median(times)
    cpu_name = ''
    try:
        for line in open('/proc/cpuinfo'):
            if line.startswith('model name'):
                cpu_name = line.split(':', 1)[1].strip()
                break
    except OSError:
        pass
    return {'value': round(batch / dt, 4), 'unit': 'pairs/s', 'cores': threads, 'kind': 'port',
            'sample': f'contrastive step (fwd+bwd+clip+Adam), base config, batch {batch}, 128-token text, fp32 '
                      f'eager oracle on CPU ({cpu_name}, {threads} threads of {os.cpu_count()} logical CPUs'
                      f'{" -- capped by " + " and ".join(caps) if caps else ""}): '
                      f'1 warm-up ({warm:.1f} s) then median of {runs} steps '
                      f'({", ".join(f"{t:.1f}" for t in times)} s)',
            'step_s_median': round(dt, 3), 'step_s_runs': [round(t, 3) for t in times]}


def _cgroup_cpus():
    """CPUs of this process's cgroup quota (cgroup v2 cpu.max / v1 cfs), or None if unlimited."""
    try:
        q, per = open('/sys/fs/cgroup/cpu.max').read().split()[:2]
        if q != 'max':
            return max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    try:
        q = int(open('/sys/fs/cgroup/cpu/cpu.cfs_quota_us').read())
        per = int(open('/sys/fs/cgroup/cpu/cpu.cfs_period_us').read())
        if q > 0:
            return max(1, q // per)
    except (OSError, ValueError):
        pass
    try:
        return len(os.sched_getaffinity(0)) if len(os.sched_getaffinity(0)) < (os.cpu_count() or 0) else None
    except (AttributeError, OSError):
        return None


def rocprof_avg_ms(key):
    """(avg_ms, calls, source) of the kernel whose name contains `key` in the rocprofv3 kernel-trace
    summary that profiles/LATEST_ROCPROF names (tools/prof_bench.sh output committed under
    profiles/), or (None, None, None)."""
    try:
        name = open(os.path.join(REPO, 'profiles', 'LATEST_ROCPROF')).read().strip()
        for line in open(os.path.join(REPO, 'profiles', name)):
            if key in line:
                f = line.split()
                return float(f[-2]) / 1e3, int(f[-4]), 'profiles/' + name
    except (OSError, ValueError, IndexError):
        pass
    return None, None, None


PMC_TAG = 'r06v'   # tools/pmc_gemm.sh <shape> <tag> on the current tree -> profiles/pmc_<tag>_<shape>.json


def pmc_record(shape, kernel_key):
    """The committed counter record (profiles/pmc_<PMC_TAG>_<shape>.json) if it belongs to the kernel
    named by kernel_key, with its path as '_src'; else None."""
    path = os.path.join(REPO, 'profiles', f'pmc_{PMC_TAG}_{shape}.json')
    try:
        rec = json.load(open(path))
    except (OSError, ValueError):
        return None
    if not any(kernel_key in k for k in rec.get('kernel', [])):
        return None
    rec['_src'] = f'profiles/pmc_{PMC_TAG}_{shape}.json'
    return rec


def launch_ranks(args):
    """``--gpus N`` (N > 1) without a torch.distributed launcher around us: start N ranks with
    torch.distributed.run (one process per GPU) as a CHILD process, before this process touches
    the GPU, and exit with its status."""
    import socket
    import subprocess
    ndev = torch.cuda.device_count()          # does not initialise the GPU
    if args.dist_backend == 'nccl' and ndev < args.gpus:
        sys.exit(f'bench.py: --gpus {args.gpus} needs {args.gpus} visible GPUs for RCCL, found {ndev} '
                 f'(--dist-backend gloo rehearses N ranks on fewer GPUs)')
    with socket.socket() as s_:
        s_.bind(('127.0.0.1', 0))
        port = s_.getsockname()[1]
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={args.gpus}',
           '--master-addr', '127.0.0.1', f'--master-port={port}', os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')
    sys.exit(subprocess.run(cmd, env=env).returncode)


def main():
    args = parse()
    if args.batch is None:
        args.batch = 16 if args.fp8 else 8
    if args.gpus > 1 and 'WORLD_SIZE' not in os.environ:
        launch_ranks(args)
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world != args.gpus:
        sys.exit(f'bench.py: WORLD_SIZE {world} != --gpus {args.gpus}')
    dev = torch.device('cuda', local % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    if world > 1:
        if args.dist_backend == 'nccl':
            dist.init_process_group('nccl', device_id=dev)
        else:
            dist.init_process_group('gloo')
        if dist.get_world_size() != args.gpus:
            sys.exit(f'bench.py: process group has {dist.get_world_size()} ranks, --gpus {args.gpus}')

    from ctclip_mi355x.models import build_ctclip, set_finetune_trainable
    from ctclip_mi355x.trainer import CTClipTrainer
    from ctclip_mi355x import kernels as K

    if args.fp8:
        from ctclip_mi355x import functional as Fn
        Fn.set_vit_fp8(True)
    if args.f32_tower:
        args.vit_precision = 'f32'
    if args.vit_precision and args.vit_precision != 'bf16':
        from ctclip_mi355x import precise
        precise.set_vit_precision(args.vit_precision)
        args.no_precise = True
        args.f32_tower = True   # (labels: the image-tower forward is the precise one)
    torch.manual_seed(0)   # identical random-init weights on every rank
    model = set_finetune_trainable(build_ctclip()).to(dev)
    model.train()
    # the text bucket's Adam queued by the next step's forward (trainer.defer_text_adam); flushed
    # after the warm-up (untimed) and after the last timed step (timed), so the timed region holds
    # exactly K steps' work.  CTCLIP_DEFER_TEXT_ADAM=0: queued at the end of its own step (A/B)
    trainer = CTClipTrainer(model, defer_text_adam=os.environ.get('CTCLIP_DEFER_TEXT_ADAM', '0') != '0')
    hu, text = synthetic_inputs(args.batch, args.text_len, rank, dev)

    # live timing of the dominant kernel + the ViT forward (HIP events on the launch stream)
    vt = model.visual_transformer
    orig_encode = vt.encode_pooled
    vit_events = []

    def timed_encode(video):
        if K.TIMER.active:
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            out = orig_encode(video)
            e.record()
            vit_events.append((s, e))
            return out
        return orig_encode(video)
    vt.encode_pooled = timed_encode

    for _ in range(args.warmup):
        trainer.train_step(text, hu)
    trainer.flush()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    K.TIMER.start(['ff1', 'dw', 'patch_ln'])
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = trainer.train_step(text, hu)
    trainer.flush()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    K.TIMER.stop()
    loss_v = float(loss.item())
    # every warm-up and timed step's LayerNorm-exchange status was checked by the trainer (before
    # the f32-mode steps below add theirs)
    ln_checked = trainer.ln_steps_checked
    precise_entries = {}
    modes = {
        # the SURVEY 8(c) contract modes (precise.py): the loss the step differentiates from an
        # f32-accurate image-tower forward, bf16 backward; same workload, after the timed region
        'split': "precise.set_vit_precision('split'): split-fp16 x3 GEMMs (fp16 hi / lo operand pairs, three "
                 "fp16 MFMA products per K-step into f32) + f32 PEG / LayerNorm / cosine attention image-tower "
                 "forward, bf16 backward; 0 VQ flips above the 1e-6 margin at configs[1] (test_gpu_base.py)",
        'f32': "precise.set_vit_precision('f32'): exact-f32 image-tower forward (f32 MFMA GEMMs, f32 PEG / "
               "LayerNorm / cosine attention), bf16 backward",
    }
    for mode in (() if args.no_precise or args.fp8 else ('split', 'f32')):
        from ctclip_mi355x import precise
        with precise.vit_precision_scope(mode):
            for _ in range(2):
                trainer.train_step(text, hu)
            trainer.flush()
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize()
            n_p = 5
            t1 = time.perf_counter()
            for _ in range(n_p):
                lp = trainer.train_step(text, hu)
            trainer.flush()
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize()
            el_p = time.perf_counter() - t1
        if world > 1:
            t = torch.tensor([el_p], device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el_p = t.item()
        precise_entries[mode] = {'value': round(world * args.batch * n_p / el_p, 3), 'unit': 'pairs/s',
                                 'steps': n_p, 'warmup': 2, 'ms_per_step': round(1000 * el_p / n_p, 3),
                                 'vs_bf16_step': round(el_p / n_p / (elapsed / args.steps), 3),
                                 'loss': round(float(lp.item()), 5), 'mode': modes[mode]}
    # the eval-mode 3D-ViT forward (zero-shot inference / VisionFeatureExtractor): encode + VQ + pool +
    # projection under no_grad, no backward-only tensors written (functional.ViTLayerFn lean path)
    vit_eval_ms = None
    if not args.fp8 and not args.no_eval_forward:
        model.eval()
        W = model.to_visual_latent.weight
        with torch.no_grad():
            for _ in range(2):
                model._project(W, model._visual_weight_bf16(W), *vt.encode_pooled(hu))
            torch.cuda.synchronize()
            s_ev, e_ev = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s_ev.record()
            for _ in range(5):
                model._project(W, model._visual_weight_bf16(W), *orig_encode(hu))
            e_ev.record()
            torch.cuda.synchronize()
        vit_eval_ms = s_ev.elapsed_time(e_ev) / 5
        model.train()
    if world > 1:
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    # every rank must hold identical parameters (one SUM all-reduce of identical-order buckets)
    in_sync = None
    if world > 1:
        ck = trainer.flat.data.double().sum().reshape(1)
        lo, hi = ck.clone(), ck.clone()
        dist.all_reduce(lo, op=dist.ReduceOp.MIN)
        dist.all_reduce(hi, op=dist.ReduceOp.MAX)
        in_sync = bool(lo.item() == hi.item())
    ff1 = K.TIMER.summary('ff1')
    dw = K.TIMER.summary('dw')
    pln = K.TIMER.summary('patch_ln')
    vit_ms = sum(s.elapsed_time(e) for s, e in vit_events) / max(1, len(vit_events))

    pairs = world * args.batch * args.steps
    value = pairs / elapsed
    result = {
        'metric': 'CT-report pairs/sec (contrastive step)',
        'value': round(value, 3),
        'unit': 'pairs/s',
        'n_gpus': world,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': round(1000 * elapsed / args.steps, 3),
        'higher_is_better': True,
        'scaling': 'weak',
        'vs_baseline': None,
        'dtype': 'mx-fp8 e4m3 (3D-ViT forward linears) + bf16' if args.fp8 else
                 (f'{args.vit_precision} image-tower forward + bf16 backward' if args.f32_tower else 'bf16'),
        'data': 'synthetic: int16 HU volumes 1x240x480x480 (randint -1200..1200) + 128-token reports; '
                'random-init CT-CLIP base weights',
        'config': {'workload': 'CT-CLIP base contrastive train step: BERT-base(128 tok, train-mode dropout '
                               '0.1) + CTViT(480^2x240, patch 20x20x10, 4+4 layers, VQ 8192) + InfoNCE + bwd + RCCL grad all-reduce + '
                               'clip 0.5 + Adam',
                   'per_gpu_batch': args.batch, 'global_batch': world * args.batch, 'text_len': args.text_len,
                   'parallelism': f'dp{world}', 'infonce_negatives': 'global batch (RCCL all-gather)',
                   **({'precision': 'configs[3]: Q / KV / attn-out / FF1+GEGLU / FF2 forward GEMMs MX-fp8 '
                                    '(e4m3, e8m0 per 32 k), backward bf16'} if args.fp8 else {})},
        'loss': round(loss_v, 5),
    }
    # the LayerNorm-fused GEMMs' in-launch tile-pair exchange never timed out: the trainer's own
    # per-step check of ctclip_gemm_ln's status word (a timeout raises LayerNormExchangeError in
    # train_step / flush and its step's Adam update is skipped on the device)
    result['ln_exchange_ok'] = ln_checked == args.warmup + args.steps
    result['ln_exchange_steps_checked'] = ln_checked
    if 'split' in precise_entries:
        result['precise_split_tower'] = precise_entries['split']
    if 'f32' in precise_entries:
        result['precise_f32_tower'] = precise_entries['f32']
    if in_sync is not None:
        result['ranks_in_sync'] = in_sync
        result['dist'] = {'backend': dist.get_backend(), 'world_size': dist.get_world_size(),
                          'devices_visible': torch.cuda.device_count()}
    if args.dist_backend != 'nccl':
        result['note'] = f'{args.dist_backend} rehearsal: {world} ranks on {torch.cuda.device_count()} GPU(s)'
    # kernel names in the rocprof summary / counter records: the 8-phase kernel's fourth template
    # argument is its fp16-operand flag (the default 3D-ViT forward, functional.vit_f16, round 5)
    from ctclip_mi355x import functional as Fn
    h16 = (Fn.vit_f16() and Fn._LN1_FOLD and Fn._PEG_X32 and not args.fp8 and not args.f32_tower)
    # (the fifth template argument: the split-fp16 x3 kernels, round 6; the default step runs X3 = false)
    ff1_key = f'gemm8p_kernel<true, true, 2, {"true" if h16 else "false"}, false>'
    ff1_shape = 'ff1h16' if h16 else 'ff1'
    dw_key = 'gemm8p_kernel<false, false, -5, false, false>'
    if ff1:
        tflops = ff1['flops'] / (ff1['avg_ms'] * 1e-3) / 1e12
        M = args.batch * 24 * 24 * 24
        algo_bytes = 2 * (M * 512 + 2816 * 512 + M * (2816 + 1408))   # A + W1 + h + GEGLU(h), bf16
        # counter record of the SAME kernel (tools/pmc_gemm.sh ff1 -> tools/pmc_gemm_json.py): used only
        # when its kernel name matches the one reported here
        traffic, traffic_src, mfma_busy = None, None, None
        rec = pmc_record(ff1_shape, ff1_key) if args.batch == 8 else None
        if rec:
            traffic = round(rec['traffic_bytes_per_launch'] / 1e9, 4)
            mfma_busy = round(rec['mfma_busy'], 4)
            traffic_src = (f'{rec["_src"]} (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE per launch; '
                           'mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / SIMD-cycles)')
        result['roofline'] = {
            'kernel': f'g256::{ff1_key} FF1 (LN-out x W1^T, GEGLU epilogue'
                      f'{", fp16 operands and h" if h16 else ""})',
            'bound': 'mfma', 'achieved': round(tflops, 1), 'peak': PEAK_BF16_TFLOPS, 'unit': 'TFLOP/s',
            'frac': round(tflops / PEAK_BF16_TFLOPS, 4), 'traffic': traffic, 'traffic_unit': 'GB',
            'traffic_source': traffic_src, 'mfma_busy': mfma_busy, 'algorithmic_bytes': algo_bytes,
            'hbm_frac': round(algo_bytes / (ff1['avg_ms'] * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
            'avg_launch_ms': round(ff1['avg_ms'], 4), 'flops_per_launch': ff1['flops'],
            'launches': ff1['launches'], 'timing': 'HIP events around each launch on its stream, timed region'}
        # headline = this run's HIP-event average (the contract's clock); the committed rocprofv3
        # summary's average for the same kernel is the cross-check beside it (rocprof_*, and the
        # ratio of the two: the profiled run's slower host shifts the text stream's overlap)
        result['roofline']['frac_source'] = 'live'
        rp_ms, rp_calls, rp_src = rocprof_avg_ms(ff1_key)
        if rp_ms and args.batch == 8:
            rtf = ff1['flops'] / (rp_ms * 1e-3) / 1e12
            result['roofline'].update({
                'live_achieved': round(tflops, 1), 'live_frac': round(tflops / PEAK_BF16_TFLOPS, 4),
                'rocprof_avg_launch_ms': round(rp_ms, 4), 'rocprof_achieved': round(rtf, 1),
                'rocprof_frac': round(rtf / PEAK_BF16_TFLOPS, 4),
                'rocprof_over_live': round(rp_ms / ff1['avg_ms'], 3),
                'rocprof_source': f'{rp_src} ({rp_calls} launches)'})
    if dw:
        # the kernel with the largest share of the step's time (rocprof): the split-K weight-gradient
        # GEMM, 33 launches per step of five shapes (3D-ViT Q | K | V / attention-out / FF1 / FF2 dW per
        # layer + the patch-embed dW); achieved = their algorithmic flops / their summed durations
        tf = dw['total_flops'] / (dw['total_ms'] * 1e-3) / 1e12
        rec = pmc_record('dwtn', dw_key) if args.batch == 8 else None
        # FF1-shape dW launch (2816 x 512 x 110592): algorithmic = dy + x bf16 reads + 11 f32 split-K
        # slabs (kernels.matmul_tn: 256 // 22 tiles)
        dw_algo = 2 * (args.batch * 13824 * (2816 + 512)) + 4 * 2816 * 512 * 11
        result['roofline_dominant'] = {
            'kernel': f'g256::{dw_key} split-K weight-gradient GEMMs (all launches of a step)',
            'bound': 'mfma', 'achieved': round(tf, 1), 'peak': PEAK_BF16_TFLOPS, 'unit': 'TFLOP/s',
            'frac': round(tf / PEAK_BF16_TFLOPS, 4),
            'traffic': round(rec['traffic_bytes_per_launch'] / 1e9, 4) if rec else None, 'traffic_unit': 'GB',
            'traffic_scope': 'the FF1-shape launch (2816x512x110592, split-K 11 slabs)' if rec else None,
            'traffic_algorithmic': round(dw_algo / 1e9, 4),
            'mfma_busy_ff1_shape': round(rec['mfma_busy'], 4) if rec else None,
            'mfma_busy_source': f'{rec["_src"]} (the 2816x512x110592 launch)' if rec else None,
            'avg_launch_ms': round(dw['total_ms'] / dw['launches'], 4),
            'launches_per_step': round(dw['launches'] / args.steps, 2),
            'flops_per_step': round(dw['total_flops'] / args.steps)}
        rp_ms, rp_calls, rp_src = rocprof_avg_ms(dw_key)
        # the rocprof average only prices this launch mix when the summary holds whole steps of it
        # (a summary of an older tree with another launch count per step would mis-state the frac)
        per_step = dw['launches'] // args.steps
        if rp_ms and args.batch == 8 and per_step and rp_calls % per_step:
            result['roofline_dominant']['rocprof_skipped'] = (
                f'{rp_src}: {rp_calls} launches is not a whole number of steps of {per_step}')
            rp_ms = None
        if rp_ms and args.batch == 8:
            avg_flops = dw['total_flops'] / dw['launches']
            rtf = avg_flops / (rp_ms * 1e-3) / 1e12
            result['roofline_dominant'].update({'frac_source': 'live', 'live_achieved': round(tf, 1),
                                                'live_frac': round(tf / PEAK_BF16_TFLOPS, 4),
                                                'rocprof_avg_launch_ms': round(rp_ms, 4),
                                                'rocprof_achieved': round(rtf, 1),
                                                'rocprof_frac': round(rtf / PEAK_BF16_TFLOPS, 4),
                                                'rocprof_over_live': round(rp_ms / (dw['total_ms'] / dw['launches']), 3),
                                                'rocprof_source': f'{rp_src} ({rp_calls} launches)'})
    if vit_ms > 0:
        vit_tf = VIT_FWD_GFLOP_PER_VOL * args.batch / (vit_ms * 1e-3) / 1e3
        result['vit_forward'] = {'ms': round(vit_ms, 3), 'achieved_tflops': round(vit_tf, 1),
                                 'frac_of_bf16_peak': round(vit_tf / PEAK_BF16_TFLOPS, 4),
                                 'gflop_per_volume': VIT_FWD_GFLOP_PER_VOL}
    if pln:
        result['patch_ln_in_step'] = {'avg_ms': round(pln['avg_ms'], 4), 'launches': pln['launches'],
                                      'timing': 'HIP events around the patch LayerNorm on the main stream, '
                                                'timed steps (beside whatever the other streams run)'}
    if vit_eval_ms:
        ev_tf = VIT_FWD_GFLOP_PER_VOL * args.batch / (vit_eval_ms * 1e-3) / 1e3
        result['vit_forward_eval'] = {'ms': round(vit_eval_ms, 3), 'achieved_tflops': round(ev_tf, 1),
                                      'frac_of_bf16_peak': round(ev_tf / PEAK_BF16_TFLOPS, 4),
                                      'batch': args.batch, 'scope': 'model.eval(), no_grad: encode + VQ + pool + '
                                      'image projection (HIP events, 5 calls after 2 warm-up)'}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        del trainer, model
        torch.cuda.empty_cache()
        result['cpu_baseline'] = cpu_baseline(args.cpu_batch)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
