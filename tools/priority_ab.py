"""Do HIP stream priorities shorten the bench step?  BERT (text stream) runs beside the 3D-ViT (the
critical path) and slows it through shared CUs; a higher-priority queue for the image tower (or a
lower one for BERT) lets the dispatcher prefer the ViT's workgroups.  Runs bench.py's configs[1]
train step in one process under each setting, interleaved rounds, and prints the median ms/step.
usage: python tools/priority_ab.py [steps]   (GPU)"""
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'ctpa-clip_amd'))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    from ctclip_mi355x.models import build_ctclip, set_finetune_trainable
    from ctclip_mi355x import trainer as T, streams
    dev = torch.device('cuda', 0)
    print('torch.cuda.Stream.priority_range():', torch.cuda.Stream.priority_range(), flush=True)
    lo, hi = torch.cuda.Stream.priority_range()     # (least, greatest): greatest is the smallest number
    torch.manual_seed(0)
    model = set_finetune_trainable(build_ctclip()).to(dev)
    tr = T.CTClipTrainer(model)
    hu, text = bench.synthetic_inputs(8, 128, 0, dev)
    text_default = streams.text_stream(dev)
    confs = {
        'default': (None, text_default),
        'main high': (torch.cuda.Stream(dev, priority=hi), text_default),
        'main high, text low': (torch.cuda.Stream(dev, priority=hi), torch.cuda.Stream(dev, priority=lo)),
        'text high (control)': (None, torch.cuda.Stream(dev, priority=hi)),
    }
    res = {k: [] for k in confs}

    def run(main_s, text_s, n):
        streams._STREAMS[0] = text_s
        ctx = torch.cuda.stream(main_s) if main_s is not None else torch.cuda.stream(torch.cuda.current_stream())
        with ctx:
            torch.cuda.current_stream().wait_stream(torch.cuda.default_stream())
            for _ in range(2):
                tr.train_step(text, hu)
            tr.flush()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(n):
                tr.train_step(text, hu)
            tr.flush()
            torch.cuda.synchronize()
            return 1e3 * (time.perf_counter() - t0) / n

    for rnd in range(3):
        for k, (m, t) in confs.items():
            res[k].append(run(m, t, steps))
        print(f'round {rnd}: ' + ', '.join(f'{k} {v[-1]:.2f}' for k, v in res.items()), flush=True)
    streams._STREAMS[0] = text_default
    print('median ms/step over 3 interleaved rounds:')
    for k, v in res.items():
        print(f'  {k:22s} {statistics.median(v):8.3f}')


if __name__ == '__main__':
    main()
