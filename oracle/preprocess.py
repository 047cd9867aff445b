"""CPU restatement of the reference's CT volume preprocessing — TEST INFRASTRUCTURE ONLY
(the checker for ctclip_mi355x.preprocess / libctclip_hip ctclip_resample_volume; the product
never imports this module).

  * ``npz_to_tensor``: ``ct_clip/data.py:114-192`` (CTReportDataset.npz_img_to_tensor after its
    metadata-CSV lookup, which supplies slope / intercept / spacings as arguments here), with
    ``resize_array`` of ``data.py:15-40``;
  * ``offline``: ``data_prep/preprocess_train.py:67-104`` (process_file between reading the NIfTI
    and saving the npz), with its ``resize_array`` (``:31-42``, identical to data.py's).

numpy promotion is part of the arithmetic being restated: ``slope * scan + intercept`` is f64
for integer / f64 scans and f32 for f32 scans, and ``F.interpolate`` then runs in that dtype.
Pinned by tests/golden/golden_preprocess.safetensors (make_golden_preprocess.py runs the
reference's own npz_img_to_tensor and resize_array)."""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

TARGET_SPACING = (1.5, 0.75, 0.75)      # (z, x, y): data.py:134-136, preprocess_train.py:89-91
TARGET_SHAPE = (480, 480, 240)          # (h, w, d): data.py:155


def resize(vol_dhw: torch.Tensor, current, target=TARGET_SPACING):
    """resize_array (data.py:15-40): trilinear, align_corners=False, to int(n * cur / tgt)."""
    size = [int(vol_dhw.shape[i] * (current[i] / target[i])) for i in range(3)]
    return F.interpolate(vol_dhw[None, None], size=size, mode='trilinear', align_corners=False)[0, 0].numpy()


def _window(n, t):
    """Centre crop bounds along one axis (data.py:159-161)."""
    s = max((n - t) // 2, 0)
    return s, min((n - t) // 2 + t, n)


def npz_to_tensor(scan: np.ndarray, slope, intercept, xy_spacing, z_spacing, target_shape=TARGET_SHAPE):
    """arr_0 (axes as stored) -> (1, d, h, w) f32 in [-1, 1], pad value -1."""
    v = slope * scan + intercept
    v = np.transpose(v, (2, 0, 1))
    r = resize(torch.tensor(v), (z_spacing, xy_spacing, xy_spacing))
    r = np.transpose(r, (1, 2, 0))
    r = (np.clip(r, -1000, 1000) / 1000).astype(np.float32)
    (h0, h1), (w0, w1), (d0, d1) = (_window(n, t) for n, t in zip(r.shape, target_shape))
    r = torch.tensor(r)[h0:h1, w0:w1, d0:d1]
    pads = []
    for ax in (2, 1, 0):                 # F.pad order: last axis first (data.py:165-189)
        gap = target_shape[ax] - r.shape[ax]
        pads += [gap // 2, gap - gap // 2]
    r = F.pad(r, pads, value=-1)
    return r.permute(2, 0, 1).unsqueeze(0)


def offline(img: np.ndarray, slope, intercept, xy_spacing, z_spacing):
    """NIfTI data (axes as read) -> resized (d, h, w) f32 as saved to the npz."""
    v = slope * img + intercept
    v = (np.clip(v, -1000, 1000) / 1000).astype(np.float32)
    v = v.transpose(2, 0, 1)
    return resize(torch.tensor(v), (z_spacing, xy_spacing, xy_spacing))
