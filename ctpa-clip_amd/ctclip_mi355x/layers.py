"""Host-side layout helpers shared by the model modules."""
from __future__ import annotations

import torch


def patch_offsets(C, PT, P, F, H, W):
    """Voxel offset of patch element e = ((c*PT + pt)*P + p1)*P + p2 from the patch origin, i.e. the
    '(c pt p1 p2)' order of ``Rearrange('b c (t pt) (h p1) (w p2) -> b t h w (c pt p1 p2)')``
    (ct_clip/ctvit.py:170).  int32 [C*PT*P*P]."""
    c = torch.arange(C).view(C, 1, 1, 1)
    pt = torch.arange(PT).view(1, PT, 1, 1)
    p1 = torch.arange(P).view(1, 1, P, 1)
    p2 = torch.arange(P).view(1, 1, 1, P)
    off = c * (F * H * W) + pt * (H * W) + p1 * W + p2
    return off.reshape(-1).to(torch.int32)
