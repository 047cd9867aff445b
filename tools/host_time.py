"""Host-side enqueue time of the contrastive step vs its GPU time (is the step host-bound?).
usage: python tools/host_time.py [steps]   (GPU)"""
import os
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
    from ctclip_mi355x.trainer import CTClipTrainer
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    model = set_finetune_trainable(build_ctclip()).to(dev)
    tr = CTClipTrainer(model)
    hu, text = bench.synthetic_inputs(8, 128, 0, dev)
    for _ in range(3):
        tr.train_step(text, hu)
    torch.cuda.synchronize()
    ev = lambda: torch.cuda.current_stream().record_event(torch.cuda.Event(enable_timing=True))  # noqa: E731
    from ctclip_mi355x import streams
    ts = streams.text_stream(dev)
    mark = torch.cuda.Stream(dev)   # idle stream: an event on it completes when the host queues it
    tev = lambda s: s.record_event(torch.cuda.Event(enable_timing=True))  # noqa: E731
    for _ in range(steps):
        t0 = time.perf_counter()
        e0 = ev()
        model.train()
        model.defer_text_backward = True
        loss = model(text, hu, device=dev, return_loss=True)
        e1 = ev()
        g_tf = tev(ts)
        h_f = tev(mark)
        t1 = time.perf_counter()
        loss.backward()
        e2 = ev()
        t2 = time.perf_counter()
        h_tb = tev(mark)
        d, model._deferred_text = model._deferred_text, None
        t_raw, leaf, tev_ready = d
        ts.wait_event(tev_ready)
        g_tb0 = tev(ts)
        leaf.grad.record_stream(ts)
        with torch.cuda.stream(ts):
            torch.autograd.backward(t_raw, leaf.grad)
        g_tb1 = tev(ts)
        model.defer_text_backward = False
        t3 = time.perf_counter()
        tr.optimizer_step()
        e4 = ev()
        g_ta = tev(ts)
        t4 = time.perf_counter()
        torch.cuda.synchronize()
        t5 = time.perf_counter()
        print(f'host: fwd {1e3 * (t1 - t0):6.1f} ms  vit bwd {1e3 * (t2 - t1):6.1f}  text bwd {1e3 * (t3 - t2):6.1f}  '
              f'opt {1e3 * (t4 - t3):6.1f}  | main stream: fwd {e0.elapsed_time(e1):6.1f}  bwd {e1.elapsed_time(e2):6.1f}  '
              f'opt(+text join) {e2.elapsed_time(e4):6.1f}  | step wall {1e3 * (t5 - t0):6.1f} ms', flush=True)
        print(f'  gpu clock from step start: host queued fwd by {e0.elapsed_time(h_f):6.1f}, text bwd at '
              f'{e0.elapsed_time(h_tb):6.1f} | text stream: fwd done {e0.elapsed_time(g_tf):6.1f}, bwd '
              f'{e0.elapsed_time(g_tb0):6.1f} .. {e0.elapsed_time(g_tb1):6.1f} | main bwd done {e0.elapsed_time(e2):6.1f}, '
              f'step done {e0.elapsed_time(e4):6.1f}, text Adam done {e0.elapsed_time(g_ta):6.1f}',
              flush=True)


if __name__ == '__main__':
    main()
