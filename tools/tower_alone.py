"""How much does the text tower cost inside the overlapped step?  Times, at configs[1] (B = 8):
the full train step; the 3D-ViT alone (encode + visual projection, backward of a scalar of the
latents; no BERT); BERT alone (forward + backward of a scalar of the CLS latents), each on the
main stream with nothing beside it.   usage: python tools/tower_alone.py (GPU); TOWER_ONLY=bert: BERT alone only (for rocprofv3)"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'ctpa-clip_amd'))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import bench  # noqa: E402
from ctclip_mi355x.models import build_ctclip, set_finetune_trainable  # noqa: E402
from ctclip_mi355x.trainer import CTClipTrainer  # noqa: E402
from ctclip_mi355x import functional as Fn  # noqa: E402


def timeit(fn, n=8):
    for _ in range(3):
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
    model = set_finetune_trainable(build_ctclip()).to(dev)
    model.train()
    tr = CTClipTrainer(model)
    hu, text = bench.synthetic_inputs(8, 128, 0, dev)
    if os.environ.get('TOWER_ONLY') != 'bert':
        full = timeit(lambda: tr.train_step(text, hu))

    def vit():
        pooled, pooled_b = model.visual_transformer.encode_pooled(hu)
        W = model.to_visual_latent.weight
        i_raw = model._project(W, model._visual_weight_bf16(W), pooled, pooled_b)
        i_raw.float().square().sum().backward()

    def bert():
        enc = model.text_transformer(text.input_ids, attention_mask=text.attention_mask)[0]
        t_raw = Fn.TextProjFn.apply(enc[:, 0, :].contiguous(), model.to_text_latent.weight)
        t_raw.float().square().sum().backward()
        torch.cuda.current_stream().wait_stream(torch.cuda.current_stream())
    if os.environ.get('TOWER_ONLY') == 'bert':      # for a rocprofv3 kernel trace of BERT alone
        timeit(bert, n=5)
        torch.cuda.synchronize()
        return
    v = timeit(vit)
    b = timeit(bert)
    torch.cuda.synchronize()
    print(f'full step {full:.2f} ms | 3D-ViT fwd+bwd alone {v:.2f} ms | BERT fwd+bwd alone {b:.2f} ms | '
          f'full - ViT alone = {full - v:.2f} ms (BERT + loss + optimizer inside the overlapped step)', flush=True)


if __name__ == '__main__':
    main()
