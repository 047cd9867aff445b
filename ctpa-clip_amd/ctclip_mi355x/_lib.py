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
LIB_PATH = os.path.join(_HERE, 'libctclip_hip.so')
_LIB = None

c_i64 = ctypes.c_int64
c_i32 = ctypes.c_int32
c_f32 = ctypes.c_float
c_vp = ctypes.c_void_p


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
    ]


# name -> argtypes (restype is always int32)
_SIGS = {
    'ctclip_version': [],
    'ctclip_device_arch': [ctypes.c_char_p, c_i32],
    'ctclip_gemm': [ctypes.POINTER(GemmArgs), c_vp],
    'ctclip_reduce_slabs': [c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, c_i64, c_i32, c_i32, c_vp],
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
        for name, argtypes in _SIGS.items():
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
