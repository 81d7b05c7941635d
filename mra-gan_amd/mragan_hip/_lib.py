"""ctypes binding of libmragan_hip.so (C ABI declared in include/mragan_hip.h).

The library is the only compute path of this package: there is no CPU or eager-PyTorch
fallback.  If the shared object is missing, `lib()` raises; if a kernel call returns a
non-zero status, the wrapper raises RuntimeError with the library's message.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import torch  # noqa: F401  (torch must be loaded first: the .so resolves libamdhip64 against torch's copy)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MRAGAN_HIP_LIB", os.path.join(os.path.dirname(_HERE), "lib", "libmragan_hip.so"))

ABI_VERSION = 19

vp = C.c_void_p
i32 = C.c_int
i64 = C.c_int64
f32 = C.c_float
sz = C.c_size_t

# name -> (restype, argtypes)
SIGNATURES = {
    "mragan_abi_version": (i32, []),
    "mragan_last_error": (C.c_char_p, []),
    "mragan_set_conv_precision": (i32, [i32]),
    "mragan_get_conv_precision": (i32, []),
    "mragan_set_loss_scale": (i32, [f32]),
    "mragan_get_loss_scale": (f32, []),
    "mragan_conv3d_fwd": (i32, [vp, i32, i32, i32, i32, i32, vp, vp, i32, i32, i32, i32, i32, vp, i32, i32, i32, vp, sz,
                                vp]),
    "mragan_conv3d_transposed": (i32, [vp, i32, i32, i32, i32, i32, vp, vp, i32, i32, i32, i32, i32, vp, i32, i32, i32,
                                       vp, sz, vp]),
    "mragan_conv3d_presplit": (i32, [vp, i32, i32, i32, i32, i32, vp, vp, vp, i32, i32, i32, i32, i32, vp, i32, i32,
                                     i32, i32, vp, sz, vp]),
    "mragan_conv3d_workspace": (sz, [i32] * 13),
    "mragan_conv3d_wgrad_workspace": (sz, [i32, i32, i32, i32, i32, i32, i32, i32]),
    "mragan_conv3d_wgrad": (i32, [vp, i32, i32, i32, i32, i32, vp, i32, i32, i32, i32, i32, i32, i32, vp, i32, vp, sz, vp]),
    "mragan_pack_weight": (i32, [vp, i32, i32, i32, i32, vp, vp]),
    "mragan_pack_entry_size": (sz, []),
    "mragan_pack_weights": (i32, [vp, i32, i64, vp]),
    "mragan_instnorm_workspace": (sz, [i32, i32, i32, i32, i32]),
    "mragan_instnorm_fwd": (i32, [vp, i32, i32, i32, i32, i32, vp, i32, i32, vp, i32, vp, vp, vp, sz, vp]),
    "mragan_instnorm_bwd": (i32, [vp, vp, vp, i32, i32, i32, i32, i32, vp, i32, vp, i32, vp, vp, sz, vp]),
    "mragan_conv3d_presplit_in_stats": (i32, [vp, i32, i32, i32, i32, i32, vp, vp, vp, i32, i32, i32, i32, i32, vp, i32,
                                              i32, i32, i32, vp, sz, vp, sz, vp, vp]),
    "mragan_instnorm_fwd_partials": (i32, [vp, i32, i32, i32, i32, i32, vp, i32, i32, vp, i32, vp, vp, vp, i32, vp]),
    "mragan_instnorm_bwd_g": (i32, [vp, vp, vp, i32, i32, i32, i32, i32, vp, i32, vp, i32, vp, vp, vp, sz, vp]),
    "mragan_instnorm_running_update": (i32, [vp, i32, f32, vp]),
    "mragan_running_entry_size": (sz, []),
    "mragan_rpad": (i32, [vp, i32, i32, i32, i32, i32, i32, vp, vp]),
    "mragan_rpad_fold": (i32, [vp, i32, i32, i32, i32, i32, i32, vp, vp, vp]),
    "mragan_act_bwd": (i32, [vp, vp, vp, vp, i64, i32, vp, vp]),
    "mragan_channel_concat": (i32, [vp, i32, i32, vp, i32, i32, i64, vp, vp]),
    "mragan_channel_split": (i32, [vp, i32, i32, i64, vp, i32, vp, vp, i32, vp, vp]),
    "mragan_l1_loss": (i32, [vp, vp, i64, f32, vp, i32, vp, i32, vp, vp]),
    "mragan_gan_loss": (i32, [vp, i64, f32, i32, f32, vp, i32, vp, vp, vp]),
    "mragan_channel_sum_workspace": (sz, [i64, i32]),
    "mragan_channel_sum": (i32, [vp, i64, i32, vp, i32, vp, sz, vp]),
    "mragan_adam": (i32, [vp, vp, vp, vp, i64, f32, f32, f32, f32, i32, f32, vp]),
    "mragan_adam_hyper": (i32, [f32, f32, f32, f32, i32, f32, vp]),
    "mragan_adam_dev": (i32, [vp, vp, vp, vp, i64, vp, vp]),
    "mragan_adam_dev_checked": (i32, [vp, vp, vp, vp, i64, vp, vp, vp]),
    "mragan_nonfinite_flag": (i32, [vp, i64, vp, vp]),
    "mragan_skip_count": (i32, [vp, vp, vp]),
    "mragan_adam_rebias": (i32, [vp, vp, vp, vp]),
    "mragan_fill": (i32, [vp, i64, f32, vp]),
    "mragan_debug_stamps": (i32, [vp, i32]),
    "mragan_launch_log": (C.c_char_p, [i32]),
    "mragan_crop_patches": (i32, [vp, i32, i32, i32, vp, i32, i32, i32, i32, vp, vp]),
    "mragan_patch_gather": (i32, [vp, i32, i32, i32, vp, i32, i32, i32, i32, vp, vp]),
    "mragan_patch_combine": (i32, [vp, i32, i32, i32, i32, i32, i32, i32, i32, vp, vp]),
    # ABI 11: 16-bit operand planes (bf16 / fp16 modes)
    "mragan_instnorm_fwd_op16": (i32, [vp, i32, i32, i32, i32, i32, vp, vp, i32, i32, vp, i32, vp, vp, vp, sz, vp]),
    "mragan_instnorm_fwd_partials_op16": (i32, [vp, i32, i32, i32, i32, i32, vp, vp, i32, i32, vp, i32, vp, vp, vp, i32,
                                                vp]),
    "mragan_instnorm_bwd_op16": (i32, [vp, vp, vp, i32, i32, i32, i32, i32, vp, i32, vp, i32, vp, vp, vp, sz, vp]),
    "mragan_conv3d_op16": (i32, [vp, i32, i32, i32, i32, i32, vp, vp, i32, i32, i32, i32, vp, i32, i32, i32, i32, vp, sz,
                                 vp, sz, vp, vp]),
    "mragan_conv3d_wgrad_op16": (i32, [vp, i32, i32, i32, i32, i32, vp, i32, i32, i32, i32, i32, i32, i32, vp, i32, vp,
                                       sz, vp]),
    # ABI 14: stride-2 weight gradient with a 16-bit gathered operand
    "mragan_conv3d_wgrad_g16": (i32, [vp, i32, i32, i32, i32, i32, vp, i32, i32, i32, i32, i32, i32, i32, vp, i32, vp,
                                      sz, vp]),
    "mragan_conv3d_op16_dgrad_in_stats": (i32, [vp, i32, i32, i32, i32, i32, vp, vp, i32, vp, vp, sz, vp, vp, vp, i32,
                                                vp, sz, vp, vp]),
    "mragan_instnorm_bwd_partials_op16": (i32, [vp, vp, vp, i32, i32, i32, i32, i32, vp, i32, vp, i32, vp, vp, vp, i32,
                                                vp, sz, vp]),
    # ABI 15: InstanceNorm statistics finalized in the producing conv, apply-only IN passes
    "mragan_conv3d_op16_fin": (i32, [vp, i32, i32, i32, i32, i32, vp, vp, i32, i32, i32, i32, vp, i32, i32, i32, i32, vp,
                                     sz, vp, sz, vp, vp, vp, vp, vp, vp]),
    "mragan_conv3d_op16_dgrad_in_stats_fin": (i32, [vp, i32, i32, i32, i32, i32, vp, vp, i32, vp, vp, sz, vp, vp, vp,
                                                    i32, vp, sz, vp, vp, vp, vp, vp]),
    # ABI 18: the ResnetBlock skip gradient joining the data-gradient epilogue's backward statistics
    "mragan_conv3d_op16_dgrad_in_stats_add": (i32, [vp, i32, i32, i32, i32, i32, vp, vp, i32, vp, vp, sz, vp, vp, vp,
                                                    i32, vp, vp, sz, vp, vp, vp, vp, vp]),
    "mragan_instnorm_apply_op16": (i32, [vp, i32, i32, i32, i32, i32, vp, vp, i32, i32, vp, i32, vp, vp, vp]),
    "mragan_instnorm_bwd_apply_op16": (i32, [vp, vp, vp, i32, i32, i32, i32, i32, vp, i32, vp, i32, vp, vp, vp, vp]),
    # ABI 16: the stride-2 data gradient with backward statistics on the plane of its input
    "mragan_conv3d_op16_bwd_stats": (i32, [vp, i32, i32, i32, i32, i32, vp, i32, i32, i32, i32, vp, i32, i32, i32, i32,
                                           vp, sz, vp, vp, vp, i32, vp, sz, vp, vp]),
    # ABI 17: the k7 layers on 16-bit operand planes
    "mragan_conv3d_thin_op16": (i32, [vp, i32, i32, i32, i32, i32, vp, vp, i32, i32, i32, i32, i32, vp, i32, i32, i32,
                                      i32, vp, sz, vp]),
    "mragan_conv3d_wgrad_thin_op16": (i32, [vp, i32, i32, i32, i32, i32, vp, i32, i32, i32, i32, i32, i32, i32, vp, i32,
                                            vp, sz, vp]),
    # ABI 12: the G head's data gradient with the backward statistics of the IN in front of it
    "mragan_conv3d_dgrad_in_stats": (i32, [vp, i32, i32, i32, i32, i32, vp, i32, i32, vp, vp, sz, vp, vp, vp, i32, i32,
                                           vp, sz, vp, vp]),
    "mragan_instnorm_bwd_partials": (i32, [vp, vp, vp, i32, i32, i32, i32, i32, vp, i32, vp, i32, vp, vp, vp, i32, vp, sz,
                                           vp]),
    # ABI 19: the interior + shell data-gradient rule as a query
    "mragan_conv3d_dgrad_split": (i32, [i32] * 6),
    "mragan_conv3d_wgrad_op16_pair": (i32, [vp, i32, vp, vp, i32, vp] + [i32] * 11 + [vp, i32, vp, sz, vp]),
    "mragan_conv3d_presplit_bwd_stats": (i32, [vp, i32, i32, i32, i32, i32, vp, vp, i32, i32, i32, i32, vp, i32, i32, i32,
                                               i32, vp, sz, vp, vp, vp, i32, vp, sz, vp, vp]),
}

_lock = threading.Lock()
_lib = None


class MraganError(RuntimeError):
    pass


def lib():
    """Load (once) and return the ctypes library handle.  Raises if it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise MraganError(f"libmragan_hip.so not found at {LIB_PATH}: build it with "
                              f"`python mra-gan_amd/build.py` (or __graft_entry__.build())")
        h = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(h, name)
            fn.restype = res
            fn.argtypes = args
        v = h.mragan_abi_version()
        if v != ABI_VERSION:
            raise MraganError(f"libmragan_hip ABI {v} != expected {ABI_VERSION}")
        _lib = h
    return _lib


def exported_symbols():
    return list(SIGNATURES)


def call(name: str, *args):
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        msg = lib().mragan_last_error().decode(errors="replace")
        raise MraganError(f"{name} failed (status {rc}): {msg}")
    return rc


def query(name: str, *args):
    return getattr(lib(), name)(*args)
