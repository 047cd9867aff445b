"""Golden vectors for the volume preprocessing, produced by the
REFERENCE's own code on CPU.  Run in the build container only (needs /root/reference):
    python tests/golden/make_golden_preprocess.py

  * online: ``CTReportDataset.npz_img_to_tensor`` (ct_clip/data.py:114-192) called as is on
    synthetic npz files; its metadata CSV read (pd.read_csv of a hard-coded path) is answered
    with a one-row frame carrying the case's slope / intercept / spacings;
  * offline: data_prep/preprocess_train.py's own ``resize_array`` (nibabel, absent offline, is
    stubbed at import; process_file itself writes to a hard-coded folder and deletes its input,
    so its three arithmetic lines before the resize are restated: oracle/preprocess.offline).

The fixture stores inputs, parameters and the non-padding window of each output (the rest of
the 240 x 480 x 480 tensor is the pad value -1; the window offsets are stored too)."""
from __future__ import annotations

import os
import sys
import tempfile
import types

import numpy as np
import pandas as pd
import torch
from safetensors.torch import save_file

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden  # noqa: E402  (stubs + reference path)

CASES = [
    # name, scan dtype, arr_0 shape, slope, intercept, xy, z
    ('i16', np.int16, (24, 20, 190), 1.0, -1024.0, 0.8, 2.0),      # d cropped 253 -> 240, h / w padded
    ('f32', np.float32, (20, 22, 60), 0.5, -1000.5, 0.7, 1.2),     # all axes padded, f32 arithmetic
]
OFFLINE = ('f64', (20, 18, 40), 1.0, -1024.0, 0.9, 2.5)


def _scan(dtype, shape, seed):
    g = np.random.default_rng(seed)
    if dtype == np.int16:
        return g.integers(-1200, 2600, size=shape).astype(np.int16)
    return (g.random(shape) * 3800 - 1200).astype(dtype)


def main():
    make_golden.install_stubs()
    sys.path.insert(0, make_golden.REF)
    import ct_clip.data as D
    out = {}
    with tempfile.TemporaryDirectory() as tmp:
        for k, (name, dt, shape, slope, icpt, xy, z) in enumerate(CASES):
            scan = _scan(dt, shape, 10 + k)
            path = os.path.join(tmp, f'case_{name}.npz')
            np.savez(path, scan)
            meta = pd.DataFrame({'VolumeName': [f'case_{name}.nii'], 'RescaleSlope': [slope],
                                 'RescaleIntercept': [icpt], 'XYSpacing': [f'[{xy}, {xy}]'], 'ZSpacing': [z]})
            D.pd = types.SimpleNamespace(read_csv=lambda *a, **kw: meta)
            t = D.CTReportDataset.npz_img_to_tensor(types.SimpleNamespace(split='train'), path, None)
            t = t[0]                                   # (240, 480, 480)
            keep = (t != -1).nonzero()
            lo, hi = keep.min(0).values, keep.max(0).values + 1
            win = t[lo[0]:hi[0], lo[1]:hi[1], lo[2]:hi[2]].contiguous()
            assert int((t != -1).sum()) <= win.numel()
            out[f'{name}.scan'] = torch.from_numpy(scan)
            out[f'{name}.params'] = torch.tensor([slope, icpt, xy, z], dtype=torch.float64)
            out[f'{name}.window_lo'] = lo.to(torch.int64)
            out[f'{name}.window'] = win
            out[f'{name}.sum'] = t.double().sum().reshape(1)
            print(name, tuple(t.shape), 'window', lo.tolist(), hi.tolist())
    sys.modules['nibabel'] = types.ModuleType('nibabel')
    sys.path.insert(0, os.path.join(os.path.dirname(make_golden.REF), 'CTPA_CLIP', 'data_prep'))
    import preprocess_train as PT
    name, shape, slope, icpt, xy, z = OFFLINE
    img = np.random.default_rng(20).random(shape) * 3800 - 1200        # get_fdata -> f64
    v = (np.clip(slope * img + icpt, -1000, 1000) / 1000).astype(np.float32).transpose(2, 0, 1)
    r = PT.resize_array(torch.tensor(v)[None, None], (z, xy, xy), (1.5, 0.75, 0.75))[0][0]
    out['off.img'] = torch.from_numpy(img)
    out['off.params'] = torch.tensor([slope, icpt, xy, z], dtype=torch.float64)
    out['off.resized'] = torch.from_numpy(np.ascontiguousarray(r))
    print('offline', r.shape)
    path = os.path.join(HERE, 'golden_preprocess.safetensors')
    save_file(out, path, metadata={'generator': 'tests/golden/make_golden_preprocess.py',
                                   'reference': 'sharonct/CTPA-CLIP @ 2025-06-20 (ct_clip/data.py:15-192, '
                                                'data_prep/preprocess_train.py:31-104)'})
    print('->', path)


if __name__ == '__main__':
    main()
