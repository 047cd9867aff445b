"""Is the contrastive step host-bound?  After warm-up, K train_step calls are queued without any
sync: host_ms = wall time per step until the host has queued all K, gpu_ms = wall time per step
until the device finishes.  host_ms well below gpu_ms: the GPU never waits for the host (at least
on average; the per-step maximum lead is (gpu_ms - host_ms) * K).  usage: python tools/host_ahead.py [K]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'ctpa-clip_amd'))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    from ctclip_mi355x.models import build_ctclip, set_finetune_trainable
    from ctclip_mi355x.trainer import CTClipTrainer
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    model = set_finetune_trainable(build_ctclip()).to(dev)
    tr = CTClipTrainer(model)
    hu, text = bench.synthetic_inputs(8, 128, 0, dev)
    for _ in range(3):
        tr.train_step(text, hu)
    torch.cuda.synchronize()
    marks = []
    t0 = time.perf_counter()
    for _ in range(K):
        tr.train_step(text, hu)
        marks.append(time.perf_counter())
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    per = [1e3 * (b - a) for a, b in zip([t0] + marks[:-1], marks)]
    print(f'host queue {1e3 * (t1 - t0) / K:.2f} ms/step (per call: {", ".join(f"{x:.1f}" for x in per)}) | '
          f'GPU {1e3 * (t2 - t0) / K:.2f} ms/step', flush=True)


if __name__ == '__main__':
    main()
