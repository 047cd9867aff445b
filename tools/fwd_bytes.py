"""Run 3 contrastive train steps at configs[1] (B = 8) for a PMC pass (tools/fwd_bytes.sh): the last
step's 3D-ViT forward is then summarised per kernel by tools/fwd_bytes_table.py.   (GPU)"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'ctpa-clip_amd'))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import bench  # noqa: E402
from ctclip_mi355x.models import build_ctclip, set_finetune_trainable  # noqa: E402
from ctclip_mi355x.trainer import CTClipTrainer  # noqa: E402


def main():
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    model = set_finetune_trainable(build_ctclip()).to(dev)
    model.train()
    tr = CTClipTrainer(model)
    hu, text = bench.synthetic_inputs(8, 128, 0, dev)
    for _ in range(3):
        tr.train_step(text, hu)
    tr.flush()
    torch.cuda.synchronize()
    print('done', flush=True)


if __name__ == '__main__':
    main()
