"""CT volume preprocessing on the GPU — the loader arithmetic the
reference runs per sample on the host, as one HIP launch (``ctclip_resample_volume``):

  * ``ct_volume_to_tensor``: ``ct_clip/data.py:114-192`` (CTReportDataset.npz_img_to_tensor
    after its metadata lookup) — rescale, trilinear resize to 1.5 x 0.75 x 0.75 mm
    (``resize_array``, data.py:15-40), clip to [-1000, 1000] HU, / 1000, centre crop / pad
    (value -1) to 480 x 480 x 240, returned as the (1, D, H, W) f32 tensor CTViT consumes;
  * ``preprocess_offline``: ``data_prep/preprocess_train.py:67-104`` (process_file) — rescale,
    clip, / 1000, f32, resize; returns the (D, H, W) volume the script saves as npz.

The geometry (resized extents, crop window, padding) is computed here with Python's own float
and floor-division semantics, exactly as the reference computes it; the kernel reads the scan
through strides, so the (axis 2, 0, 1) transpose of data.py:139 costs nothing.
"""
from __future__ import annotations

import ctypes

import torch

from ._lib import call, ptr, stream_ptr, ResampleArgs

TARGET_SPACING = (1.5, 0.75, 0.75)      # (z, x, y): data.py:134-136, preprocess_train.py:89-91
TARGET_SHAPE = (480, 480, 240)          # (h, w, d): data.py:155

_DT = {torch.float32: 0, torch.int16: 1, torch.float64: 2}


def resized_shape(shape_dhw, current_spacing, target_spacing=TARGET_SPACING):
    """``resize_array``'s size (data.py:27-33): int(n * (current / target)) per axis."""
    return [int(shape_dhw[i] * (current_spacing[i] / target_spacing[i])) for i in range(3)]


def crop_pad(n, t):
    """One axis of data.py:159-176 for a resized extent n and target t: (crop start, pad before)."""
    start = max((n - t) // 2, 0)
    kept = min((n - t) // 2 + t, n) - start
    return start, (t - kept) // 2


def _args(scan, dhw_axes, slope, intercept, Dn, Hn, Wn, Do, Ho, Wo, od, oh, ow, mode, fill):
    if not scan.is_cuda:
        raise ValueError('preprocess: the scan must be a device tensor')
    if scan.dtype not in _DT:
        raise ValueError(f'preprocess: unsupported scan dtype {scan.dtype}')
    a = ResampleArgs()
    a.src, a.src_dtype = ptr(scan), _DT[scan.dtype]
    d, h, w = dhw_axes
    a.D, a.H, a.W = scan.shape[d], scan.shape[h], scan.shape[w]
    a.sd, a.sh, a.sw = scan.stride(d), scan.stride(h), scan.stride(w)
    a.Dn, a.Hn, a.Wn = Dn, Hn, Wn
    a.Do, a.Ho, a.Wo = Do, Ho, Wo
    a.od, a.oh, a.ow = od, oh, ow
    a.slope, a.intercept = float(slope), float(intercept)
    a.mode, a.fill = mode, fill
    return a


def ct_volume_to_tensor(scan, slope, intercept, xy_spacing, z_spacing, target_shape=TARGET_SHAPE, out=None):
    """``arr_0`` of a preprocessed npz (device tensor, axes as stored; data.py reads them as
    (h, w, d)) -> (1, D, H, W) f32 in [-1, 1] with pad value -1."""
    if scan.ndim != 3:
        raise ValueError(f'preprocess: expected a 3-D scan, got {tuple(scan.shape)}')
    d, h, w = 2, 0, 1                                   # np.transpose(img, (2, 0, 1)), data.py:139
    Dn, Hn, Wn = resized_shape((scan.shape[d], scan.shape[h], scan.shape[w]), (z_spacing, xy_spacing, xy_spacing))
    th, tw, td = target_shape
    (hs, hp), (ws, wp), (ds, dp) = crop_pad(Hn, th), crop_pad(Wn, tw), crop_pad(Dn, td)
    if out is None:
        out = torch.empty(1, td, th, tw, device=scan.device, dtype=torch.float32)
    a = _args(scan, (d, h, w), slope, intercept, Dn, Hn, Wn, td, th, tw, dp - ds, hp - hs, wp - ws, 0, -1.0)
    call('ctclip_resample_volume', ctypes.byref(a), ptr(out), stream_ptr())
    return out


def preprocess_offline(img, slope, intercept, xy_spacing, z_spacing):
    """NIfTI voxel data (device tensor, axes as ``get_fdata`` returns them) -> the resized
    (D, H, W) f32 volume of preprocess_train.py:98-104."""
    if img.ndim != 3:
        raise ValueError(f'preprocess: expected a 3-D volume, got {tuple(img.shape)}')
    d, h, w = 2, 0, 1                                   # img_data.transpose(2, 0, 1), :100
    Dn, Hn, Wn = resized_shape((img.shape[d], img.shape[h], img.shape[w]), (z_spacing, xy_spacing, xy_spacing))
    out = torch.empty(Dn, Hn, Wn, device=img.device, dtype=torch.float32)
    a = _args(img, (d, h, w), slope, intercept, Dn, Hn, Wn, Dn, Hn, Wn, 0, 0, 0, 1, 0.0)
    call('ctclip_resample_volume', ctypes.byref(a), ptr(out), stream_ptr())
    return out


__all__ = ['ct_volume_to_tensor', 'preprocess_offline', 'resized_shape', 'crop_pad', 'TARGET_SHAPE',
           'TARGET_SPACING']
