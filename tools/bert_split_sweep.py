"""Text-tower precision vs cost of the hi / lo split BERT weights, per number of split layers
(CTCLIP_TEXT_SPLIT_LAYERS): text latents and logits (oracle forced onto the HIP VQ indices) against
the reference's base fixture (golden_base_b2), as in tests/test_gpu_base.py.  GPU."""
import math
import os
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'ctpa-clip_amd'))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from safetensors.torch import load_file  # noqa: E402

from oracle import ctclip_oracle as O  # noqa: E402
from oracle import weights as W  # noqa: E402
from ctclip_mi355x import functional as Fn  # noqa: E402


def main():
    from test_gpu_model import build
    torch.set_num_threads(16)
    CFG = O.BASE
    g = load_file(os.path.join(ROOT, 'tests', 'golden', 'golden_base_b2.safetensors'))
    sd = W.make_state_dict(CFG)
    model = build(CFG)
    model.eval()
    hu = W.make_hu(2, CFG.vit)
    ids, mask = W.make_text(2, 128, CFG.bert.vocab_size)
    text = types.SimpleNamespace(input_ids=ids.cuda(), attention_mask=mask.cuda())
    e = math.e
    forced = None
    for k in (12, 8, 6, 4, 3, 2, 1, 0):
        Fn._TEXT_SPLIT_LAYERS = k
        with torch.no_grad():
            _, _, t_raw, i_raw = model.encode(text, hu.cuda())
            idx = model.visual_transformer.vq.state.last_indices.cpu()
        torch.cuda.synchronize()
        if forced is None:
            with torch.no_grad():
                forced = O.ctclip_forward(sd, ids, mask, O.normalize_hu(hu), CFG, training=False, force_ind=idx)
        tl, il = F.normalize(t_raw, dim=-1).cpu(), F.normalize(i_raw, dim=-1).cpu()
        dt = (tl - g['out.text_latents']).abs().max().item()
        flog = (tl @ il.t() * e - forced['text_latents'] @ forced['image_latents'].t() * e).abs().max().item()
        print(f'split layers {k:2d}: text latents vs fixture {dt:.2e}, logits vs forced oracle {flog:.2e}', flush=True)


if __name__ == '__main__':
    main()
