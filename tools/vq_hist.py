"""Diagnostic: VQ code usage in the bench setting (random-init model, synthetic volumes): codes
used, top-1 / 10 / 100 counts and the fraction of consecutive token rows sharing a code -- what
decides whether the EMA statistics kernel (vq.hip) could merge rows before its atomics.
usage (GPU): python tools/vq_hist.py"""
import sys, os
sys.path.insert(0, os.path.join(os.getcwd(), 'ctpa-clip_amd')); sys.path.insert(0, os.getcwd())
import torch, bench
from ctclip_mi355x.models import build_ctclip, set_finetune_trainable
from ctclip_mi355x.trainer import CTClipTrainer
dev = torch.device('cuda', 0)
torch.manual_seed(0)
model = set_finetune_trainable(build_ctclip()).to(dev)
tr = CTClipTrainer(model)
hu, text = bench.synthetic_inputs(8, 128, 0, dev)
for i in range(3):
    tr.train_step(text, hu)
    idx = model.visual_transformer.vq.state.last_indices
    c = torch.bincount(idx.long().reshape(-1), minlength=8192).sort(descending=True).values
    n = c.sum().item()
    print(f'step {i}: rows {n}, used codes {(c > 0).sum().item()}, top1 {c[0].item()}, top10 {c[:10].sum().item()}, '
          f'top100 {c[:100].sum().item()}', flush=True)
    flat = idx.reshape(-1)
    print('  consecutive-equal fraction', (flat[1:] == flat[:-1]).float().mean().item(), flush=True)
