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
                ("n_enc", C.c_int), ("n_dec", C.c_int), ("dtype", C.c_int), ("max_batch", C.c_int),
                ("n_classes", C.c_int), ("class_dim", C.c_int)]


class CvaeLossWeights(C.Structure):
    _fields_ = [("recon", C.c_float), ("kld", C.c_float), ("start", C.c_float), ("time", C.c_float)]


class CvaeMpcConfig(C.Structure):
    _fields_ = [(k, C.c_double) for k in ("wheelbase", "max_steer", "max_accel", "dt", "q_theta", "q_v", "qf_theta",
                                          "qf_v", "r_accel", "r_steer", "tol")] + \
               [(k, C.c_int) for k in ("prediction_horizon", "control_horizon", "max_iter", "reserved")]


class CvaeAdamConfig(C.Structure):
    _fields_ = [("lr", C.c_double), ("beta1", C.c_double), ("beta2", C.c_double), ("eps", C.c_double)]


CVAE_F32, CVAE_BF16, CVAE_FP8 = 0, 1, 2
CVAE_X_OPERAND, CVAE_X_F32 = 0, 1
CVAE_PART_CHAIN, CVAE_PART_DW_DEC, CVAE_PART_DW_REST, CVAE_PART_ALL = 1, 2, 4, 7

_v, _i, _u64, _i64, _f, _d = C.c_void_p, C.c_int, C.c_uint64, C.c_int64, C.c_float, C.c_double
_W = C.POINTER(CvaeLossWeights)
_A = C.POINTER(CvaeAdamConfig)
_SIGS = {
    "cvae_create": (_i, [C.POINTER(CvaeConfig), _i, C.POINTER(_v)]),
    "cvae_destroy": (_i, [_v]),
    "cvae_num_params": (_i, [_v, c_i64p, C.POINTER(_i)]),
    "cvae_param_info": (_i, [_v, _i, c_i64p, c_i64p, C.POINTER(_i), C.POINTER(_i)]),
    "cvae_config_info": (_i, [C.POINTER(CvaeConfig), c_i64p, C.POINTER(_i), C.POINTER(_i)]),
    "cvae_workspace_bytes": (_i, [_v, c_i64p]),
    "cvae_bucket_split": (_i, [_v, c_i64p]),
    "cvae_train_kernel": (_i, [_v, C.POINTER(_i)]),
    "cvae_dw_kernel": (_i, [_v, C.POINTER(_i)]),
    "cvae_chain_rows": (_i, [_v, _i, C.POINTER(_i)]),
    "cvae_pack_weights": (_i, [_v, _v, _v]),
    # h, x, idx, classes, batch, xflags, start, eps, seed, offset, eps_row0, recon, mu, logvar, hc, eps_out, stream
    "cvae_forward": (_i, [_v, _v, _v, _v, _i, _i, _v, _v, _u64, _u64, _i64, _v, _v, _v, _v, _v, _v]),
    "cvae_condition": (_i, [_v, _v, _i, _v, _v]),
    "cvae_decode": (_i, [_v, _v, _v, _v, _v, _i, _v, _v]),  # h, z, start, hc, classes, batch, out, stream
    # h, x, idx, classes, batch, xflags, eps, seed, offset, eps_row0, w, grads, loss_out, loss_accum, counters,
    # adam, parts, stream
    "cvae_train_fwd_bwd": (_i, [_v, _v, _v, _v, _i, _i, _v, _u64, _u64, _i64, _W, _v, _v, _v, _v, _A, _i, _v]),
    # h, x, idx, classes, batch, xflags, start, eps, seed, offset, eps_row0, d_recon, d_mu, d_logvar, d_hc, grads,
    # stream
    "cvae_backward": (_i, [_v, _v, _v, _v, _i, _i, _v, _v, _u64, _u64, _i64, _v, _v, _v, _v, _v, _v]),
    # h, params, grads, m, v, step, adam, grad_scale, counters, stream
    "cvae_adam": (_i, [_v, _v, _v, _v, _v, _i64, _A, _f, _v, _v]),
    # h, params, grads (the shard), m, v, lo, count, step, adam, grad_scale, counters, stream
    "cvae_adam_flat": (_i, [_v, _v, _v, _v, _v, _i64, _i64, _i64, _A, _f, _v, _v]),
    # h, x, idx, classes, batch, xflags, eps, seed, offset, eps_row0, w, params, m, v, step, adam, loss_out,
    # loss_accum, counters, stream
    "cvae_train_step": (_i, [_v, _v, _v, _v, _i, _i, _v, _u64, _u64, _i64, _W, _v, _v, _v, _i64, _A, _v, _v, _v,
                             _v]),
    "cvae_train_steps": (_i, [_v, _v, _v, _v, _i, _i, _i, _v, _u64, _u64, _i64, _W, _v, _v, _v, _i64, _A, _v, _v,
                              _v, _v]),
    # h, x, idx, classes, n_rows, batch, n_steps, xflags, eps, seed, offset, eps_row0, w, params, m, v, step0,
    # adam, loss_out, loss_accum, counters, stream
    "cvae_train_epochs": (_i, [_v, _v, _v, _v, _i, _i, _i, _i, _v, _u64, _u64, _i64, _W, _v, _v, _v, _i64, _A, _v,
                               _v, _v, _v]),
    "cvae_bench_kernels": (_i, [_v, _v, _v, _i, _i, _v, _v, _v, _i64, C.POINTER(_f), _v]),
    "cvae_fault": (_i, [_v, C.POINTER(C.c_uint)]),
    "cvae_clear_fault": (_i, [_v]),
    "cvae_step_skip": (_i, [_v, _v, _A, _v]),  # h, counters, adam, stream
    "cvae_px_blob_bytes": (_i, [c_i64p]),
    "cvae_px_export": (_i, [_v, _i, _i, _v]),  # h, world, rank, blob
    "cvae_px_import": (_i, [_v, _v, _u64]),    # h, blobs, base
    "cvae_px_owned": (_i, [_v, _v]),           # h, mask (host uint8[n_params])
    "cvae_px_probe": (_i, [_v, C.POINTER(_i)]),
    "cvae_px_close": (_i, [_v]),
    "cvae_px_stats": (_i, [_v, C.POINTER(C.c_uint64), _i]),
    "cvae_px_layout": (_i, [_v, C.POINTER(_i), C.POINTER(_i)]),  # h, ranks_on_gpu, tile_blocks
    "cvae_px_reset": (_i, [_v, _u64]),                            # h, base
    "cvae_rccl_id_bytes": (_i, [c_i64p]),
    "cvae_rccl_unique_id": (_i, [_v]),                             # id (host bytes)
    "cvae_rccl_init": (_i, [_v, _v, _i, _i]),                      # h, id, world, rank
    "cvae_rccl_allreduce": (_i, [_v, _v, _i64, _v]),               # h, buf, count, stream
    "cvae_rccl_close": (_i, [_v]),
    "cvae_operand_checksum": (_i, [_v, _v, _v]),                  # h, out (device u64), stream
    "cvae_tap_outputs": (_i, [_v, _v, _v, _v]),                   # h, recon, mu, logvar
    "cvae_read_activation": (_i, [_v, _i, _i, _i, _v, C.POINTER(_i), _v]),  # h, layer, which, rows, dst, features, stream
    # h, x, idx, batch, xflags, eps, seed, eps_row0, w, params, m, v, adam, rank_scales, loss_out, loss_accum,
    # counters, stream
    "cvae_px_train_step": (_i, [_v, _v, _v, _i, _i, _v, _u64, _i64, _W, _v, _v, _v, _A, _v, _v, _v, _v, _v]),
    "cvae_loss": (_i, [_v, _v, _v, _v, _i, _i, _i, _i, _W, _v, _v, _v]),
    "cvae_loss_backward": (_i, [_v, _v, _v, _v, _i, _i, _i, _i, _W, _v, _v, _v, _v, _v]),
    "cvae_adam_scalars": (_i, [_A, _i64, _v, _v]),
    # cols, n_rows, file_offsets, n_files, scene, target_points, point_mode, time_interval, out, valid, stream
    "cvae_extract_trajectories": (_i, [_v, _i64, _v, _i, _i, _i, _i, _d, _v, _v, _v]),
    "cvae_mpc_default_config": (_i, [C.POINTER(CvaeMpcConfig)]),
    # cfg, n_paths, waypoints, wp_offsets, initial_states, n_steps, step_offsets, states, controls, iters, stream
    "cvae_mpc_track": (_i, [C.POINTER(CvaeMpcConfig), _i, _v, _v, _v, _v, _v, _v, _v, _v, _v]),
    # cfg, n, state, ref, last, u, cost, iters, stream
    "cvae_mpc_solve": (_i, [C.POINTER(CvaeMpcConfig), _i, _v, _v, _v, _v, _v, _v, _v]),
    # n_paths, waypoints, wp_offsets, initial_states, t, n_t, out, scalars, stream
    "cvae_mpc_reference": (_i, [_i, _v, _v, _v, _v, _i, _v, _v, _v]),
    "cvae_set_timing": (_i, [_v, _i]),
    "cvae_kernel_times": (_i, [_v, C.c_char_p, _i, C.POINTER(_f), _i]),
    "cvae_last_error": (C.c_char_p, []),
    "cvae_abi_version": (_i, []),
}
ABI_VERSION = 3

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
        if h.cvae_abi_version() != ABI_VERSION:
            raise RuntimeError(f"{LIB} has ABI {h.cvae_abi_version()}, this binding expects {ABI_VERSION} (rebuild)")
        _lib = h
    return _lib


def header_symbols(header_path: str):
    """Function names declared in include/cvae.h (used by the export test)."""
    txt = open(header_path).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(cvae_\w+)\s*\(", txt, re.M)))


def missing_signatures(header_path: str):
    """Header functions without a ctypes signature here (the binding must cover the whole ABI)."""
    return [n for n in header_symbols(header_path) if n not in _SIGS]


class CvaeError(RuntimeError):
    pass


def check(rc, what="cvae call"):
    if rc < 0:
        raise CvaeError(f"{what} failed ({rc}): {lib().cvae_last_error().decode(errors='replace')}")
    return rc


def ptr(t):
    """Device pointer of a tensor (or NULL for None)."""
    return None if t is None else C.c_void_p(t.data_ptr())
