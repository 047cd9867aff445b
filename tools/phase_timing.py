"""Wall time of the contrastive step's parts on one GPU (HIP events, median of 5):
BERT fwd, BERT fwd+bwd, CTViT fwd, CTViT fwd+bwd, full train step.  B = 8, 128 tokens."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'ctpa-clip_amd'))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from bench import synthetic_inputs  # noqa: E402
from ctclip_mi355x.models import build_ctclip, set_finetune_trainable  # noqa: E402
from ctclip_mi355x.trainer import CTClipTrainer  # noqa: E402


def timed(fn, n=5):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    return sorted(ts)[n // 2]


def main():
    dev = torch.device('cuda')
    torch.manual_seed(0)
    model = set_finetune_trainable(build_ctclip()).to(dev)
    model.train()
    tr = CTClipTrainer(model)
    hu, text = synthetic_inputs(8, 128, 0, dev)
    bert, vit = model.text_transformer, model.visual_transformer

    def bert_f():
        with torch.no_grad():
            bert(text.input_ids, attention_mask=text.attention_mask)

    def bert_fb():
        out = bert(text.input_ids, attention_mask=text.attention_mask)[0]
        out[:, 0].float().sum().backward()

    def vit_f():
        with torch.no_grad():
            vit.encode_pooled(hu)

    def vit_fb():
        pooled, _ = vit.encode_pooled(hu)
        pooled.float().sum().backward()

    rows = [('bert fwd', bert_f), ('bert fwd+bwd', bert_fb), ('vit fwd', vit_f), ('vit fwd+bwd', vit_fb),
            ('train step', lambda: tr.train_step(text, hu))]
    for name, fn in rows:
        ms = timed(fn)
        print(f'{name:14s} {ms:8.2f} ms', flush=True)
        tr.flat.grad.zero_()


if __name__ == '__main__':
    main()
