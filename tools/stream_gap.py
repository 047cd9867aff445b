"""Is there a main-stream bubble at the forward -> backward boundary of the bench step (VERDICT r03
weak 7: stream 0 idle 16.5 -> 22.9 ms in the rocprof timeline)?  Runs bench.py's configs[1] step
WITHOUT a profiler and brackets the main stream with HIP events at the phase boundaries the
trainer goes through:

    e0 step start | forward + loss | e1 | loss.backward() | e2 | host queues BERT's backward on
    the text stream | e3 | 3D-ViT backward | e4 | optimizer | e5

An event recorded on an idle stream completes when the host records it, so elapsed(e2, e3) is the
main stream's idle time while the host queues BERT's backward (0 when the host is ahead and the
image backward was already queued behind the loss).  Prints per-phase GPU ms (median over the
timed steps) and the host time of each phase.  usage: python tools/stream_gap.py [steps]"""
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
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    from ctclip_mi355x.models import build_ctclip, set_finetune_trainable
    from ctclip_mi355x import trainer as T
    from ctclip_mi355x import kernels as K
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    model = set_finetune_trainable(build_ctclip()).to(dev)
    tr = T.CTClipTrainer(model)
    hu, text = bench.synthetic_inputs(8, 128, 0, dev)
    rec = []

    def ev():
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        return e, time.perf_counter()

    def step():
        marks = [ev()]
        tr._check_ln(block_upto=tr.steps - 2)
        model.train()
        with K.ln_guard():
            tr.grad_sync.arm()
            model.defer_text_backward = True
            loss = model(text, hu, device=dev, return_loss=True)
            marks.append(ev())
            loss.backward()
            marks.append(ev())
            model.backward_deferred_text()
            marks.append(ev())
            model.backward_deferred_image()
            marks.append(ev())
            model.defer_text_backward = False
        tr.optimizer_step()
        tr._queue_ln_check()
        marks.append(ev())
        rec.append(marks)

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    rec.clear()
    for _ in range(steps):
        step()
    tr.flush()
    torch.cuda.synchronize()
    names = ['forward+loss', 'loss.backward', 'host queues BERT bwd (main-stream idle)', '3D-ViT backward',
             'optimizer']
    print(f'{steps} steps, medians (GPU ms between main-stream events | host ms between the records):')
    for i, nm in enumerate(names):
        g = statistics.median(m[i][0].elapsed_time(m[i + 1][0]) for m in rec)
        h = statistics.median(1e3 * (m[i + 1][1] - m[i][1]) for m in rec)
        print(f'  {nm:42s} GPU {g:8.3f} ms   host {h:8.3f} ms')
    tot = statistics.median(m[0][0].elapsed_time(m[-1][0]) for m in rec)
    gaps = [m[2][0].elapsed_time(m[3][0]) for m in rec]
    print(f'  step (e0 -> e5)                            GPU {tot:8.3f} ms')
    print(f'  main-stream gap per step: median {statistics.median(gaps):.3f} ms, max {max(gaps):.3f} ms')


if __name__ == '__main__':
    main()
