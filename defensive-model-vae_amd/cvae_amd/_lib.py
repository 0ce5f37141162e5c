"""ctypes binding of the C-ABI in include/cvae.h (libcvae_hip.so, built in-tree).

There is no fallback: if the library is missing or fails to load, every entry
point raises.  The product path is the HIP path.
"""
from __future__ import annotations

import ctypes as C
import os
import re

from ._build import LIB

c_i64p = C.POINTER(C.c_int64)


class CvaeConfig(C.Structure):
    _fields_ = [("seq_len", C.c_int), ("dim", C.c_int), ("latent_dim", C.c_int), ("hidden_dim", C.c_int),
                ("n_enc", C.c_int), ("n_dec", C.c_int), ("dtype", C.c_int), ("max_batch", C.c_int)]


class CvaeLossWeights(C.Structure):
    _fields_ = [("recon", C.c_float), ("kld", C.c_float), ("start", C.c_float), ("time", C.c_float)]


CVAE_F32, CVAE_BF16, CVAE_FP8 = 0, 1, 2

_SIGS = {
    "cvae_create": (C.c_int, [C.POINTER(CvaeConfig), C.c_int, C.POINTER(C.c_void_p)]),
    "cvae_destroy": (C.c_int, [C.c_void_p]),
    "cvae_num_params": (C.c_int, [C.c_void_p, c_i64p, C.POINTER(C.c_int)]),
    "cvae_param_info": (C.c_int, [C.c_void_p, C.c_int, c_i64p, c_i64p, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "cvae_config_info": (C.c_int, [C.POINTER(CvaeConfig), c_i64p, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "cvae_workspace_bytes": (C.c_int, [C.c_void_p, c_i64p]),
    "cvae_pack_weights": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    "cvae_forward": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_uint64,
                               C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "cvae_condition": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]),
    "cvae_decode": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]),
    "cvae_train_fwd_bwd": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_uint64,
                                     C.c_uint64, C.POINTER(CvaeLossWeights), C.c_void_p, C.c_void_p, C.c_void_p,
                                     C.c_void_p]),
    "cvae_adam": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_float,
                            C.c_float, C.c_float, C.c_float, C.c_float, C.c_void_p]),
    "cvae_train_step": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_uint64, C.c_uint64,
                                  C.POINTER(CvaeLossWeights), C.c_void_p, C.c_void_p, C.c_void_p, C.c_int,
                                  C.c_float, C.c_float, C.c_float, C.c_float, C.c_void_p, C.c_void_p,
                                  C.c_void_p]),
    "cvae_train_steps": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_uint64,
                                   C.c_uint64, C.POINTER(CvaeLossWeights), C.c_void_p, C.c_void_p, C.c_void_p,
                                   C.c_int, C.c_float, C.c_float, C.c_float, C.c_float, C.c_void_p, C.c_void_p,
                                   C.c_void_p]),
    "cvae_bench_kernels": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_void_p,
                                     C.c_void_p, C.c_int, C.POINTER(C.c_float), C.c_void_p]),
    "cvae_sync_words": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint)]),
    "cvae_loss": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int,
                            C.POINTER(CvaeLossWeights), C.c_void_p, C.c_void_p, C.c_void_p]),
    "cvae_set_timing": (C.c_int, [C.c_void_p, C.c_int]),
    "cvae_kernel_times": (C.c_int, [C.c_void_p, C.c_char_p, C.c_int, C.POINTER(C.c_float), C.c_int]),
    "cvae_last_error": (C.c_char_p, []),
    "cvae_abi_version": (C.c_int, []),
}

_lib = None


def lib():
    """Load libcvae_hip.so (raises if absent — there is no CPU fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            raise RuntimeError(f"HIP extension missing: {LIB} (run __graft_entry__.build())")
        h = C.CDLL(LIB)
        for name, (res, args) in _SIGS.items():
            f = getattr(h, name)
            f.restype, f.argtypes = res, args
        _lib = h
    return _lib


def header_symbols(header_path: str):
    """Function names declared in include/cvae.h (used by the export test)."""
    txt = open(header_path).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(cvae_\w+)\s*\(", txt, re.M)))


class CvaeError(RuntimeError):
    pass


def check(rc, what="cvae call"):
    if rc < 0:
        raise CvaeError(f"{what} failed ({rc}): {lib().cvae_last_error().decode(errors='replace')}")
    return rc


def ptr(t):
    """Device pointer of a tensor (or NULL for None)."""
    return None if t is None else C.c_void_p(t.data_ptr())
