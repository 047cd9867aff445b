"""Volume preprocessing (ct_clip/data.py:114-192 and
data_prep/preprocess_train.py:67-104).

CPU: the oracle restatement and the product's host-side geometry against fixtures made by the
reference's own npz_img_to_tensor / resize_array (tests/golden/make_golden_preprocess.py).
GPU: ctclip_resample_volume against the same fixtures.  Tolerances: the int16 scan runs in f64 as
numpy promotes it, so the f32 outputs are the f64 values rounded once -- bit-exact except where
the reference's CPU build rounds an intermediate differently (counted, <= 1e-4 of the voxels, each
within 1 f32 ulp); f32 scans interpolate in f32 (max |diff| 2e-6)."""
import os

import numpy as np
import pytest
import torch
from safetensors.torch import load_file

from oracle import preprocess as OP

G = load_file(os.path.join(os.path.dirname(__file__), 'golden', 'golden_preprocess.safetensors'))
CASES = ['i16', 'f32']


def _window(t, name):
    lo = G[f'{name}.window_lo'].tolist()
    w = G[f'{name}.window']
    return t[lo[0]:lo[0] + w.shape[0], lo[1]:lo[1] + w.shape[1], lo[2]:lo[2] + w.shape[2]], w


@pytest.mark.parametrize('name', CASES)
def test_oracle_online_matches_reference(name):
    slope, icpt, xy, z = G[f'{name}.params'].tolist()
    t = OP.npz_to_tensor(G[f'{name}.scan'].numpy(), slope, icpt, xy, z)[0]
    assert t.shape == (240, 480, 480) and t.dtype == torch.float32
    win, ref = _window(t, name)
    assert torch.equal(win, ref)
    # total incl. the padding (the f64 sum's order depends on the host's thread count)
    assert abs(t.double().sum().item() - G[f'{name}.sum'].item()) <= 1e-9 * abs(G[f'{name}.sum'].item())


def test_oracle_offline_matches_reference():
    slope, icpt, xy, z = G['off.params'].tolist()
    r = OP.offline(G['off.img'].numpy(), slope, icpt, xy, z)
    assert np.array_equal(r, G['off.resized'].numpy())


@pytest.mark.parametrize('name', CASES)
def test_host_geometry_matches_reference(name):
    from ctclip_mi355x.preprocess import resized_shape, crop_pad
    slope, icpt, xy, z = G[f'{name}.params'].tolist()
    H, W, D = G[f'{name}.scan'].shape
    Dn, Hn, Wn = resized_shape((D, H, W), (z, xy, xy))
    lo = G[f'{name}.window_lo'].tolist()
    ext = G[f'{name}.window'].shape
    for n, t, l0, e in zip((Dn, Hn, Wn), (240, 480, 480), lo, ext):
        start, pad = crop_pad(n, t)
        assert pad == l0 and min(n - start, t) == e


def test_crop_pad_geometry_edge_cases():
    """data.py:159-176 semantics incl. Python floor division of negative gaps."""
    from ctclip_mi355x.preprocess import crop_pad
    for n in range(1, 1200, 7):
        for t in (240, 480):
            start, pad = crop_pad(n, t)
            s = max((n - t) // 2, 0)
            e = min((n - t) // 2 + t, n)
            assert start == s and pad == (t - (e - s)) // 2
            assert pad + (e - s) <= t


@pytest.mark.gpu
@pytest.mark.parametrize('name', CASES)
def test_gpu_online_matches_reference(name):
    from ctclip_mi355x.preprocess import ct_volume_to_tensor
    slope, icpt, xy, z = G[f'{name}.params'].tolist()
    scan = G[f'{name}.scan'].cuda()
    out = ct_volume_to_tensor(scan, slope, icpt, xy, z)
    torch.cuda.synchronize()
    assert out.shape == (1, 240, 480, 480)
    t = out[0].cpu()
    win, ref = _window(t, name)
    diff = (win - ref).abs()
    if name == 'i16':
        bad = (win != ref).sum().item()
        assert bad <= max(1, ref.numel() // 10000), bad
        ulp = torch.finfo(torch.float32).eps * ref.abs().clamp_min(1e-3)
        assert bool((diff <= ulp).all())
    else:
        assert diff.max().item() <= 2e-6
    # everything outside the window is the pad value
    mask = torch.ones_like(t, dtype=torch.bool)
    lo = G[f'{name}.window_lo'].tolist()
    w = G[f'{name}.window'].shape
    mask[lo[0]:lo[0] + w[0], lo[1]:lo[1] + w[1], lo[2]:lo[2] + w[2]] = False
    assert bool((t[mask] == -1).all())
    # a strided (non-contiguous) view of the same scan gives the same bits
    st = scan.permute(2, 0, 1).contiguous().permute(1, 2, 0)
    assert not st.is_contiguous()
    out2 = ct_volume_to_tensor(st, slope, icpt, xy, z)
    assert torch.equal(out, out2)


@pytest.mark.gpu
def test_gpu_offline_matches_reference():
    from ctclip_mi355x.preprocess import preprocess_offline
    slope, icpt, xy, z = G['off.params'].tolist()
    r = preprocess_offline(G['off.img'].cuda(), slope, icpt, xy, z)
    torch.cuda.synchronize()
    ref = G['off.resized']
    assert r.shape == ref.shape
    assert (r.cpu() - ref).abs().max().item() <= 2e-6


@pytest.mark.gpu
def test_gpu_full_size_scan_matches_oracle():
    """A CT-RATE-sized scan (512 x 512 x 300 int16, 0.7 mm / 1.25 mm): d cropped, h / w padded;
    checked against the oracle on a sample of planes."""
    from ctclip_mi355x.preprocess import ct_volume_to_tensor
    g = torch.Generator().manual_seed(5)
    scan = torch.randint(-1100, 2000, (512, 512, 300), generator=g, dtype=torch.int16)
    out = ct_volume_to_tensor(scan.cuda(), 1.0, -1024.0, 0.7, 1.25)[0].cpu()
    ref = OP.npz_to_tensor(scan.numpy(), 1.0, -1024.0, 0.7, 1.25)[0]
    for d in (0, 57, 119, 200, 239):
        a, b = out[d], ref[d]
        assert (a != b).sum().item() <= max(1, a.numel() // 10000)
        assert (a - b).abs().max().item() <= 1.2e-7
