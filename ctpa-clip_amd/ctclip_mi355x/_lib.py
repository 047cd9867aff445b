"""ctypes binding of libctclip_hip.so (C-ABI declared in include/ctclip_hip.h).

The product path has NO fallback: if the library is missing or a call fails, we raise.
torch is imported first so that its bundled HIP runtime (SONAME libamdhip64.so.7) is the
one the library binds to — device pointers and streams are then shared with torch.
"""
from __future__ import annotations

import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# CTCLIP_HIP_LIB: an alternative in-tree build (A/B timing in tools/); never a fallback
LIB_PATH = os.environ.get('CTCLIP_HIP_LIB') or os.path.join(_HERE, 'libctclip_hip.so')
_LIB = None

c_i64 = ctypes.c_int64
c_i32 = ctypes.c_int32
c_f32 = ctypes.c_float
c_vp = ctypes.c_void_p


class SlabJob(ctypes.Structure):
    _fields_ = [('slabs', c_vp), ('nslab', c_i64), ('cols', c_i64), ('out', c_vp), ('accumulate', c_i32),
                ('pad', c_i32)]


ABI_VERSION = 2     # CTCLIP_ABI_VERSION of include/ctclip_hip.h that the structs below mirror


class GemmArgs(ctypes.Structure):
    _fields_ = [
        ('M', c_i64), ('N', c_i64), ('K', c_i64),
        ('A', c_vp), ('lda', c_i64), ('a_kcontig', c_i32),
        ('B', c_vp), ('ldb', c_i64), ('b_kcontig', c_i32),
        ('C', c_vp), ('ldc', c_i64), ('c_f32', c_i32),
        ('C2', c_vp), ('ldc2', c_i64),
        ('bias', c_vp),
        ('R', c_vp), ('ldr', c_i64), ('r_f32', c_i32),
        ('alpha', c_f32),
        ('act', c_i32),
        ('accumulate', c_i32),
        ('split_k', c_i32),
        ('batch', c_i32),
        ('sA', c_i64), ('sB', c_i64), ('sC', c_i64), ('sC2', c_i64), ('sR', c_i64),
        ('n2', c_i32),
        ('B2', c_vp),
        ('ab_f16', c_i32),
        ('r_f16', c_i32),
        ('A_lo', c_vp), ('B_lo', c_vp),
        ('C3', c_vp), ('ldc3', c_i64),
        ('C4', c_vp), ('ldc4', c_i64),
    ]


class LnEpilogueArgs(ctypes.Structure):
    """ctclip_ln_epilogue (include/ctclip_hip.h): LayerNorm fused into an N = 512 GEMM."""
    _fields_ = [
        ('mode', c_i32),
        ('gamma', c_vp), ('beta', c_vp), ('eps', c_f32),
        ('Y', c_vp), ('ldy', c_i64),
        ('mean', c_vp), ('rstd', c_vp),
        ('X', c_vp), ('ldx', c_i64),
        ('part_gamma', c_vp), ('part_beta', c_vp),
        ('xchg', c_vp), ('epoch', ctypes.c_uint32),
        ('status', c_vp),
        ('spin_limit', ctypes.c_uint32), ('debug', c_i32),
        ('Y16', c_vp),
    ]


class MxGemmArgs(ctypes.Structure):
    _fields_ = [
        ('M', c_i64), ('N', c_i64), ('Kp', c_i64),
        ('A', c_vp), ('lda', c_i64), ('sA', c_vp),
        ('B', c_vp), ('ldb', c_i64), ('sB', c_vp),
        ('C', c_vp), ('ldc', c_i64), ('c_f32', c_i32),
        ('bias', c_vp), ('alpha', c_f32),
        ('R', c_vp), ('ldr', c_i64),
        ('C2', c_vp), ('ldc2', c_i64),
        ('act', c_i32),
    ]


class AttnArgs(ctypes.Structure):
    _fields_ = [
        ('q', c_vp), ('ldq', c_i64), ('k', c_vp), ('ldk', c_i64), ('v', c_vp), ('ldv', c_i64),
        ('o', c_vp), ('ldo', c_i64), ('dout', c_vp), ('lddo', c_i64),
        ('dq', c_vp), ('lddq', c_i64), ('dk', c_vp), ('lddk', c_i64), ('dv', c_vp), ('lddv', c_i64),
        ('lse', c_vp), ('delta', c_vp), ('bias_u', c_vp), ('dbias_u', c_vp), ('kmask', c_vp),
        ('scale', c_f32), ('L', c_i32), ('H', c_i32), ('D', c_i32), ('nseq', c_i32), ('M', c_i64),
        ('grid_h', c_i32), ('grid_w', c_i32), ('n_inner', c_i32),
        ('s_outer', c_i64), ('s_inner', c_i64), ('s_pos', c_i64),
        ('dropout_p', c_f32), ('dropout_seed', ctypes.c_uint64),
        ('dbias_ws', c_vp), ('dbias_ws_floats', c_i64),
        ('o16', c_vp),
    ]


class SgemmTnArgs(ctypes.Structure):
    """ctclip_sgemm_tn_args (include/ctclip_hip.h): the f32 image tower's exact-f32 GEMM."""
    _fields_ = [
        ('M', c_i64), ('N', c_i64), ('K', c_i64),
        ('A', c_vp), ('lda', c_i64),
        ('B', c_vp), ('ldb', c_i64),
        ('C', c_vp), ('ldc', c_i64),
        ('C2', c_vp), ('ldc2', c_i64),
        ('C3', c_vp), ('ldc3', c_i64),
        ('bias', c_vp),
        ('R', c_vp), ('ldr', c_i64),
        ('alpha', c_f32),
        ('act', c_i32),
    ]


class ResampleArgs(ctypes.Structure):
    _fields_ = [
        ('src', c_vp), ('src_dtype', c_i32),
        ('D', c_i64), ('H', c_i64), ('W', c_i64), ('sd', c_i64), ('sh', c_i64), ('sw', c_i64),
        ('Dn', c_i64), ('Hn', c_i64), ('Wn', c_i64), ('Do', c_i64), ('Ho', c_i64), ('Wo', c_i64),
        ('od', c_i64), ('oh', c_i64), ('ow', c_i64),
        ('slope', ctypes.c_double), ('intercept', ctypes.c_double),
        ('mode', c_i32), ('fill', c_f32),
    ]


# name -> argtypes (restype is always int32)
_SIGS = {
    'ctclip_version': [],
    'ctclip_device_arch': [ctypes.c_char_p, c_i32],
    'ctclip_debug_hold_cus': [c_i32, c_i64, c_i32, c_vp],
    'ctclip_gemm': [ctypes.POINTER(GemmArgs), c_vp],
    'ctclip_gemm_ln': [ctypes.POINTER(GemmArgs), ctypes.POINTER(LnEpilogueArgs), c_vp],
    'ctclip_gemm_qkv_lnfold': [ctypes.POINTER(GemmArgs), c_vp, c_vp, c_vp, c_i32, c_vp],
    'ctclip_gemm_qkv_lnfold2': [ctypes.POINTER(GemmArgs), c_vp, c_vp, c_vp, c_i32, c_i32, c_vp],
    'ctclip_pack_qkv_fold': [c_vp, c_i64, c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp,
                             c_i32, c_vp, c_vp],
    'ctclip_ln_stats_merge': [c_vp, c_i32, c_i64, c_i32, c_f32, c_vp, c_vp, c_vp],
    'ctclip_lnfold_wgrad': [c_vp, c_i64, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, c_i64, c_vp, c_vp,
                            c_i64, c_vp],
    'ctclip_gemm_lnfold_bwd': [ctypes.POINTER(GemmArgs), c_vp, c_i64, c_vp, c_vp, c_vp],
    'ctclip_l2norm_qk_bwd_fold': [c_vp, c_i64, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_i64, c_vp, c_i32, c_vp, c_vp,
                                  c_vp, c_vp, c_i32, c_vp, c_vp, c_vp],
    'ctclip_quant_mxfp8': [c_vp, c_i32, c_i64, c_i64, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp],
    'ctclip_gemm_mxfp8': [ctypes.POINTER(MxGemmArgs), c_vp],
    'ctclip_gemm_mxfp8_set_tile': [c_i32],
    'ctclip_dropout': [c_vp, c_vp, c_vp, c_vp, c_i64, c_f32, ctypes.c_uint64, c_vp],
    'ctclip_gemm_set_variant': [c_i32],
    'ctclip_gemm_set_stagger': [c_i32],
    'ctclip_gemm_set_epi_lds': [c_i32],
    'ctclip_gemm_set_persist': [c_i32],
    'ctclip_gemm_set_grid_cap': [c_i32],
    'ctclip_reduce_slabs_ep': [c_vp, c_i64, c_i64, c_i64, c_i64, ctypes.POINTER(GemmArgs), c_vp],
    'ctclip_reduce_slabs_ep_drop': [c_vp, c_i64, c_i64, c_i64, c_i64, ctypes.POINTER(GemmArgs), c_f32, ctypes.c_uint64,
                                    c_vp],
    'ctclip_layernorm_bwd_drop': [c_vp, c_i32, c_i64, c_vp, c_i32, c_i64, c_vp, c_vp, c_vp, c_i64, c_i32, c_vp, c_i64,
                                  c_vp, c_i64, c_vp, c_vp, c_vp, c_i32, c_f32, ctypes.c_uint64, c_vp],
    'ctclip_patch_ln_x2': [c_vp, c_i32, c_i32, c_i64, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_vp, c_f32, c_vp,
                           c_vp, c_i64, c_vp],
    'ctclip_patch_ln_x3': [c_vp, c_i32, c_i32, c_i64, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_vp, c_f32, c_vp,
                           c_vp, c_vp, c_i64, c_vp],
    'ctclip_layernorm_fwd_x2': [c_vp, c_i32, c_i64, c_i64, c_i32, c_vp, c_vp, c_f32, c_vp, c_vp, c_i64, c_vp, c_i64,
                                c_vp, c_vp, c_vp],
    'ctclip_layernorm_fwd_x3': [c_vp, c_i32, c_i64, c_i64, c_i32, c_vp, c_vp, c_f32, c_vp, c_vp, c_vp, c_i64, c_vp,
                                c_i64, c_vp, c_vp, c_vp, c_vp],
    'ctclip_pack_rows_h16': [c_vp, c_i64, c_vp, c_i64, c_i32, c_i32, c_vp, c_vp, c_i64, c_vp],
    'ctclip_pack_qkv_fold_h16': [c_vp, c_i64, c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_vp, c_i64, c_vp, c_vp],
    'ctclip_skinny_gemm_slices': [c_i64, c_i64, c_i64],
    'ctclip_skinny_gemm': [c_vp, c_i64, c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, c_i32, c_vp],
    'ctclip_vq_l2norm_h16': [c_vp, c_i64, c_i64, c_i32, c_vp, c_i64, c_vp],
    'ctclip_skinny_sgemm_slices': [c_i64, c_i64, c_i64],
    'ctclip_skinny_sgemm': [c_vp, c_i64, c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, c_i32, c_vp],
    'ctclip_reduce_slabs': [c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, c_i64, c_i32, c_i32, c_vp],
    'ctclip_reduce_slabs_multi': [ctypes.POINTER(SlabJob), c_i32, c_vp],
    'ctclip_layernorm_fwd': [c_vp, c_i32, c_i64, c_i64, c_i32, c_vp, c_vp, c_f32, c_vp, c_i64, c_vp, c_i64,
                             c_vp, c_vp, c_vp],
    'ctclip_layernorm_bwd': [c_vp, c_i32, c_i64, c_vp, c_i32, c_i64, c_vp, c_vp, c_vp, c_i64, c_i32, c_vp, c_i64,
                             c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_i32, c_vp],
    'ctclip_l2norm_scale_fwd': [c_vp, c_i64, c_i64, c_i32, c_i32, c_vp, c_vp, c_i64, c_vp],
    'ctclip_l2norm_scale_bwd': [c_vp, c_i64, c_vp, c_i64, c_i64, c_i32, c_i32, c_vp, c_vp, c_i64, c_vp, c_i32, c_vp],
    'ctclip_l2norm_scale_bwd_fold': [c_vp, c_i64, c_vp, c_i64, c_i64, c_i32, c_i32, c_vp, c_vp, c_i64, c_vp, c_i32,
                                     c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_i32, c_vp, c_vp, c_vp],
    'ctclip_colsum': [c_vp, c_i32, c_i64, c_i64, c_i32, c_vp, c_i32, c_vp],
    'ctclip_geglu_bwd': [c_vp, c_i64, c_vp, c_i64, c_i64, c_i32, c_vp, c_i64, c_vp],
    'ctclip_gelu_bwd': [c_vp, c_vp, c_vp, c_i64, c_vp],
    'ctclip_pack_rows': [c_vp, c_i64, c_vp, c_i64, c_i32, c_i32, c_vp, c_vp, c_i64, c_vp],
    'ctclip_pack_rows_f32': [c_vp, c_i64, c_vp, c_i64, c_i32, c_i32, c_vp, c_vp, c_i64, c_vp],
    'ctclip_split_f16': [c_vp, c_i64, c_i64, c_i32, c_f32, c_vp, c_vp, c_i64, c_vp, c_vp],
    'ctclip_pack_rows_x3': [c_vp, c_i64, c_vp, c_i64, c_i32, c_i32, c_vp, c_f32, c_vp, c_vp, c_i64, c_vp, c_vp],
    'ctclip_sgemm_tn': [ctypes.POINTER(SgemmTnArgs), c_vp],
    'ctclip_unpack_rows': [c_vp, c_i64, c_vp, c_i64, c_i32, c_vp, c_i64, c_i32, c_vp],
    'ctclip_reduce_slabs_rows': [c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, c_vp, c_i64, c_i32, c_vp],
    'ctclip_gelu_f32': [c_vp, c_vp, c_i64, c_vp],
    'ctclip_cast_f32_bf16': [c_vp, c_vp, c_i64, c_vp],
    'ctclip_cast_f32_bf16_split': [c_vp, c_vp, c_vp, c_i64, c_vp],
    'ctclip_add_f32': [c_vp, c_vp, c_vp, c_vp, c_i64, c_vp],
    'ctclip_patch_ln': [c_vp, c_i32, c_i32, c_i64, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_vp, c_f32, c_vp, c_i64,
                        c_vp],
    'ctclip_patch_wgrad': [c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_vp, c_vp, c_vp, c_i32, c_vp],
    'ctclip_unpatch_mse': [c_vp, c_i64, c_vp, c_i32, c_i32, c_i64, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_vp,
                           c_vp, c_i64, c_vp, c_vp, c_vp, c_vp],
    'ctclip_peg_fwd': [c_vp, c_vp, c_i64, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp, c_i32, c_vp, c_vp, c_vp],
    'ctclip_peg_fwd_stats': [c_vp, c_vp, c_i64, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp, c_i32, c_vp, c_vp, c_vp,
                             c_vp],
    'ctclip_peg_fwd_x32': [c_vp, c_i64, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp],
    'ctclip_peg_fwd_x32s': [c_vp, c_i64, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp,
                            c_vp, c_vp],
    'ctclip_peg_bwd_data_x32': [c_vp, c_i64, c_i32, c_i32, c_i32, c_i32, c_vp, c_i32, c_vp, c_vp, c_vp],
    'ctclip_peg_bwd_data': [c_vp, c_vp, c_i64, c_i32, c_i32, c_i32, c_i32, c_vp, c_i32, c_vp, c_vp, c_vp],
    'ctclip_peg_bwd_weight': [c_vp, c_vp, c_i64, c_i32, c_i32, c_i32, c_i32, c_i32, c_vp, c_i32, c_vp],
    'ctclip_peg_wgrad_reduce': [c_vp, c_i32, c_i32, c_vp, c_vp, c_i32, c_vp],
    'ctclip_peg_wgrad_slabs': [c_i64, c_i32, c_i32, c_i32, c_i32],
    'ctclip_peg_set_canon1': [c_i32],
    'ctclip_attn_fwd': [ctypes.POINTER(AttnArgs), c_vp],
    'ctclip_attn_bwd': [ctypes.POINTER(AttnArgs), c_vp],
    'ctclip_attn_bwd_ws_floats': [ctypes.POINTER(AttnArgs)],
    'ctclip_attn_fwd_f32': [ctypes.POINTER(AttnArgs), c_vp],
    'ctclip_attn_fwd_x3': [ctypes.POINTER(AttnArgs), c_vp, c_vp, c_vp, c_vp, c_vp],
    'ctclip_attn_set_fwd_qb': [c_i32],
    'ctclip_attn_set_fwd_smax': [c_i32],
    'ctclip_attn_set_fwd_cinit': [c_i32],
    'ctclip_patch_ln_f32': [c_vp, c_i32, c_i32, c_i64, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_vp, c_f32, c_vp,
                            c_vp, c_vp, c_i64, c_vp],
    'ctclip_peg_fwd_f32': [c_vp, c_i64, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp, c_i32, c_vp, c_vp],
    'ctclip_l2norm_scale_fwd_f32': [c_vp, c_i64, c_i64, c_i32, c_i32, c_vp, c_vp, c_i64, c_vp],
    'ctclip_l2norm_scale_fwd_f32b': [c_vp, c_i64, c_i64, c_i32, c_i32, c_vp, c_vp, c_i64, c_vp, c_i64, c_vp],
    'ctclip_geglu_f32': [c_vp, c_i64, c_i64, c_i32, c_vp, c_i64, c_vp],
    'ctclip_vq_select': [c_vp, c_vp, c_i32, c_vp, c_i64, c_i32, c_vp, c_i32, c_f32, c_vp, c_vp, c_vp],
    'ctclip_vq_select_s': [c_vp, c_vp, c_i32, c_vp, c_i64, c_i32, c_vp, c_i32, c_f32, c_vp, c_vp, c_vp, c_vp],
    'ctclip_vq_pool': [c_vp, c_vp, c_i64, c_i32, c_i32, c_i32, c_vp, c_vp, c_vp],
    'ctclip_vq_pool_bwd': [c_vp, c_i64, c_i32, c_i32, c_i32, c_vp, c_vp, c_vp],
    'ctclip_vq_gather': [c_vp, c_vp, c_i64, c_i32, c_vp, c_vp],
    'ctclip_vq_ema_accum': [c_vp, c_vp, c_i64, c_i32, c_vp, c_vp, c_vp],
    'ctclip_vq_ema_accum_sorted': [c_vp, c_vp, c_i64, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp],
    'ctclip_vq_ema_finalize': [c_vp, c_vp, c_i32, c_i32, c_f32, c_vp, c_vp, c_vp, c_vp],
    'ctclip_vq_ema_finalize_reset': [c_vp, c_vp, c_i32, c_i32, c_f32, c_vp, c_vp, c_vp, c_vp],
    'ctclip_vq_ema_finalize_guard': [c_vp, c_vp, c_i32, c_i32, c_f32, c_vp, c_vp, c_vp, c_vp, c_vp],
    'ctclip_clip_loss': [c_vp, c_vp, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp],
    'ctclip_clip_scores': [c_vp, c_vp, c_i32, c_i32, c_vp, c_vp, c_vp],
    'ctclip_zero_shot': [c_vp, c_vp, c_i32, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp],
    'ctclip_resample_volume': [ctypes.POINTER(ResampleArgs), c_vp, c_vp],
    'ctclip_sgemm': [c_i64, c_i64, c_i64, c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_vp, c_f32,
                     c_i32, c_f32, c_vp, c_i64, c_i64, c_i32, c_vp, c_i32, c_vp],
    'ctclip_embed_fwd': [c_vp, c_i64, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp],
    'ctclip_embed_bwd': [c_vp, c_i64, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp],
    'ctclip_grad_norm': [c_vp, c_i64, c_f32, c_vp, c_i32, c_vp, c_vp],
    'ctclip_grad_norm_s': [c_vp, c_i64, c_f32, c_vp, c_i32, c_vp, c_vp, c_vp],
    'ctclip_adam': [c_vp, c_vp, c_vp, c_vp, c_i64, c_f32, c_f32, c_f32, c_f32, c_f32, c_i32, c_vp, c_vp, c_vp, c_i32,
                    c_vp, c_vp],
}


def register(name, argtypes):
    _SIGS[name] = argtypes
    if _LIB is not None:
        fn = getattr(_LIB, name)
        fn.argtypes = argtypes
        fn.restype = c_i32


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f'ctclip_mi355x: HIP library not built ({LIB_PATH}); run '
                               '`python -c "import __graft_entry__ as g; g.build()"` from the repo root')
        _LIB = ctypes.CDLL(LIB_PATH)
        # the structs below mirror include/ctclip_hip.h of ABI version ABI_VERSION: a library of
        # another version reads (or misses) trailing struct fields, so it is refused outright
        _LIB.ctclip_version.restype = c_i32
        v = _LIB.ctclip_version()
        if v != ABI_VERSION and 'CTCLIP_HIP_LIB' not in os.environ:
            _LIB = None
            raise RuntimeError(f'ctclip_mi355x: {LIB_PATH} has ABI version {v}, this binding needs '
                               f'{ABI_VERSION} (rebuild: `make -C ctpa-clip_amd/csrc`)')
        # an A/B library named by CTCLIP_HIP_LIB may predate entry points added since; those are
        # skipped (calling one fails).  The in-tree library must export every one.
        ab = 'CTCLIP_HIP_LIB' in os.environ
        for name, argtypes in _SIGS.items():
            if ab and not hasattr(_LIB, name):
                continue
            fn = getattr(_LIB, name)
            fn.argtypes = argtypes
            fn.restype = c_i32
    return _LIB


class KernelError(RuntimeError):
    pass


def call(name, *args):
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        raise KernelError(f'{name} failed with code {rc}')


def stream_ptr():
    return torch.cuda.current_stream().cuda_stream


def ptr(t):
    return None if t is None else t.data_ptr()
