"""GPU box diagnostic (round 6): the training steps of test_train_step_bit_reproducible with every
vq_assign call checked on the host -- finite tokens, finite codebook, finite candidate scores, and
the f32 argmax of the rows vq_select could not assign.  Prints one line per call."""
import os
import sys
import types

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..', 'ctpa-clip_amd'))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..', 'tests'))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..'))
from ctclip_mi355x import functional as Fn, kernels as K  # noqa: E402
from oracle import ctclip_oracle as O, weights as W  # noqa: E402

orig = Fn.vq_assign
calls = [0]


def probe(zf, zb, cb, state, want_xn=False):
    if os.environ.get('PROBE_SYNC', '1') == '0':
        return orig(zf, zb, cb, state, want_xn)
    D, C = zf.shape[1], cb.shape[0]
    nt = (C + 63) // 64
    torch.cuda.synchronize()
    zfin = torch.isfinite(zf).all().item()
    cfin = torch.isfinite(cb).all().item()
    xh = K.vq_l2norm_h16(zf)
    cbh = K.split_f16(cb)[0]
    cand = torch.empty(zf.shape[0], nt, 2, device=zf.device)
    cand2 = torch.empty(zf.shape[0], nt, device=zf.device)
    K.gemm_raw(zf.shape[0], C, D, xh, D, True, cbh, D, True, cand, nt, C2=cand2, ldc2=nt, act=K.ACT_ARGMAX)
    torch.cuda.synchronize()
    best = cand[..., 0].amax(1)
    nonf = (~torch.isfinite(best)).sum().item()
    ref = torch.nn.functional.normalize(zf, dim=-1) @ cb.t()
    rbest = ref.amax(1)
    gap = (rbest - best).abs()
    print(f'call {calls[0]}: rows {zf.shape[0]} tokens finite {zfin} codebook finite {cfin} |cb| max '
          f'{cb.abs().max().item():.3g} xh finite {torch.isfinite(xh).all().item()} cbh finite '
          f'{torch.isfinite(cbh).all().item()}; rows with non-finite best cand {nonf}; max |best - f32 best| '
          f'{gap[torch.isfinite(gap)].max().item() if torch.isfinite(gap).any() else float("nan"):.3g}; '
          f'cand2 finite frac {torch.isfinite(cand2).float().mean().item():.3f}', flush=True)
    idx, xn = orig(zf, zb, cb, state, want_xn)
    torch.cuda.synchronize()
    bad = (idx.long() != ref.argmax(1))
    print(f'   vq_assign idx differs from torch f32 argmax on {bad.sum().item()} rows; status word '
          f'{K.status_word(zf.device).item()}', flush=True)
    calls[0] += 1
    return idx, xn


Fn.vq_assign = probe


def main():
    from ctclip_mi355x.trainer import CTClipTrainer
    from test_gpu_model import build
    vit = O.ViTConfig(dim=512, codebook_size=8192, image_size=480, patch_size=20, temporal_patch_size=10,
                      spatial_depth=1, temporal_depth=1, dim_head=32, heads=8, frames=20)
    bert = O.BertConfig(vocab_size=1000, hidden=768, layers=2, heads=12, intermediate=3072, max_position=64)
    cfg = O.ClipConfig(vit=vit, bert=bert, dim_latent=512)
    torch.manual_seed(1)
    hu = W.make_hu(2, cfg.vit).cuda()
    ids, mask = W.make_text(2, 32, bert.vocab_size, ragged=True)
    text = types.SimpleNamespace(input_ids=ids.cuda(), attention_mask=mask.cuda())
    from ctclip_mi355x import ctvit, ct_clip
    cpb_aux, dema = ctvit._CPB_AUX, ct_clip.DEFER_EMA
    for run, (defer, aux, de) in enumerate(((False, cpb_aux, dema), (False, cpb_aux, dema), (True, cpb_aux, dema),
                                            (False, not cpb_aux, dema), (False, cpb_aux, '0'),
                                            (False, cpb_aux, '1'))):
        torch.manual_seed(0)
        ctvit._CPB_AUX = aux
        ct_clip.DEFER_EMA = de
        model = build(cfg, dropout=0.1)
        tr = CTClipTrainer(model, lr=1e-4, defer_text_adam=defer)
        try:
            for s in range(3):
                loss = tr.train_step(text, hu)
                print(f'run {run} step {s}: loss {loss.item():.6f}', flush=True)
            tr.flush()
        except Exception as e:  # noqa: BLE001
            print(f'run {run} ({defer}, {aux}, {de}): {type(e).__name__}: {str(e)[:120]}', flush=True)
            K.reset_ln_status()
        finally:
            ctvit._CPB_AUX = cpb_aux
            ct_clip.DEFER_EMA = dema
        torch.cuda.synchronize()

if __name__ == '__main__':
    main()
