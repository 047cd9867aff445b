"""Per-op census of one contrastive step: every top-level call into ctclip_mi355x.kernels timed
with HIP events on the stream it runs on, grouped by (op, stream, shape signature).
usage: python tools/op_census.py   (GPU)"""
import collections
import functools
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'ctpa-clip_amd'))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    from ctclip_mi355x import kernels as K
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
    rec, depth = [], [0]

    def sig(args):
        out = []
        for a in args[:3]:
            if torch.is_tensor(a):
                out.append('x'.join(map(str, a.shape)))
            elif isinstance(a, (int, float)):
                out.append(str(a))
        return ','.join(out)

    def wrap(name, fn):
        @functools.wraps(fn)
        def w(*a, **kw):
            if depth[0]:
                return fn(*a, **kw)
            st = torch.cuda.current_stream()
            e0 = st.record_event(torch.cuda.Event(enable_timing=True))
            depth[0] += 1
            try:
                return fn(*a, **kw)
            finally:
                depth[0] -= 1
                e1 = st.record_event(torch.cuda.Event(enable_timing=True))
                rec.append((name, st.stream_id != 0, sig(a), e0, e1))
        return w

    names = [n for n in dir(K) if not n.startswith('_') and callable(getattr(K, n))
             and getattr(getattr(K, n), '__module__', '') == K.__name__ and n not in ('KernelTimer', 'weights_epoch')]
    saved = {n: getattr(K, n) for n in names}
    for n in names:
        setattr(K, n, wrap(n, saved[n]))
    tr.train_step(text, hu)
    torch.cuda.synchronize()
    for n in names:
        setattr(K, n, saved[n])
    agg = collections.defaultdict(lambda: [0, 0.0])
    per_op = collections.defaultdict(lambda: [0, 0.0])
    for name, side, sg, e0, e1 in rec:
        t = e0.elapsed_time(e1)
        a = agg[(name, side, sg)]
        a[0] += 1
        a[1] += t
        b = per_op[(name, side)]
        b[0] += 1
        b[1] += t
    print('== per op (main stream first)')
    for (name, side), (n, t) in sorted(per_op.items(), key=lambda kv: (kv[0][1], -kv[1][1])):
        print(f'{"side" if side else "main"} {name:28s} {n:5d} calls {t:8.3f} ms')
    print('== per op and shape (top 60 by time)')
    for (name, side, sg), (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:60]:
        print(f'{"side" if side else "main"} {name:24s} {sg:34s} {n:4d} {t:8.3f} ms')


if __name__ == '__main__':
    main()
