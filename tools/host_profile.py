"""Where does the host spend its ~34 ms per bench step (GPU: ~40 ms)?  cProfile over the configs[1]
train step (CTClipTrainer.train_step on bench.py's synthetic batch), no GPU profiler; prints the
top functions by own time and by cumulative time.  The host queues ahead of the GPU today, so this
is the headroom check for GPU-side speedups (a step faster than the host's queueing time would be
host-bound).  usage: python tools/host_profile.py [steps]   (GPU)"""
import cProfile
import io
import os
import pstats
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'ctpa-clip_amd'))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    from ctclip_mi355x.models import build_ctclip, set_finetune_trainable
    from ctclip_mi355x import trainer as T
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    model = set_finetune_trainable(build_ctclip()).to(dev)
    tr = T.CTClipTrainer(model)
    hu, text = bench.synthetic_inputs(8, 128, 0, dev)
    for _ in range(3):
        tr.train_step(text, hu)
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    for _ in range(steps):
        tr.train_step(text, hu)
    pr.disable()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    tr.flush()
    print(f'{steps} steps: host {1e3 * (t1 - t0) / steps:.2f} ms/step under cProfile, '
          f'GPU drain after the last queue {1e3 * (t2 - t1):.1f} ms')
    for key in ('tottime', 'cumulative'):
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats(key).print_stats(35)
        print(s.getvalue())


if __name__ == '__main__':
    main()
