"""Probe: does the 3D-ViT forward gain from running two half-batches side by side on two HIP streams
(one half's HBM-bound kernels beside the other's MFMA-bound GEMMs)?  Eval mode, no grad, encoder
tokens only (no VQ / EMA state), configs[1] volumes.  Prints ms for: B = 8 on one stream; B = 4 twice
in sequence on one stream; B = 4 + 4 on two streams.
usage: python tools/mb_probe.py (GPU)"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'ctpa-clip_amd'))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import bench  # noqa: E402
from ctclip_mi355x.models import build_ctclip  # noqa: E402


def timeit(fn, n=6):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


def main():
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    model = build_ctclip().to(dev)
    model.eval()
    vit = model.visual_transformer
    hu, _ = bench.synthetic_inputs(8, 128, 0, dev)
    a, b = hu[:4].contiguous(), hu[4:].contiguous()
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    cur = torch.cuda.current_stream(dev)

    def one():
        vit.encode_tokens(hu)

    def seq():
        vit.encode_tokens(a)
        vit.encode_tokens(b)

    def two():
        ev = cur.record_event()
        s1.wait_event(ev)
        s2.wait_event(ev)
        with torch.cuda.stream(s1):
            vit.encode_tokens(a)
        with torch.cuda.stream(s2):
            vit.encode_tokens(b)
        cur.wait_stream(s1)
        cur.wait_stream(s2)

    with torch.no_grad():
        for rep in range(2):
            t1, ts, t2 = timeit(one), timeit(seq), timeit(two)
            print(f'rep {rep}: B=8 one stream {t1:.2f} ms | B=4 x2 sequential {ts:.2f} ms | '
                  f'B=4 + 4 on two streams {t2:.2f} ms ({t1 / t2:.3f}x vs B=8)', flush=True)
        # the two-stream result must equal the one-stream tokens
        za = vit.encode_tokens(a)[0].clone()
        ev = cur.record_event()
        s1.wait_event(ev)
        with torch.cuda.stream(s1):
            zb = vit.encode_tokens(a)[0]
        cur.wait_stream(s1)
        torch.cuda.synchronize()
        print('two-stream tokens equal:', bool(torch.equal(za, zb)), flush=True)


if __name__ == '__main__':
    main()
