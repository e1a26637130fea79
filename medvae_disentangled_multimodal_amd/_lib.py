"""ctypes binding of the C-ABI hot-path library (include/medvae_hip.h -> libmvae_hip.so).

There is deliberately NO fallback: if the shared library is missing or fails to load, every op
raises. The product path is the HIP path.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import c_double, c_float, c_int, c_longlong, c_size_t, c_uint64, c_void_p

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MVAE_HIP_LIB", os.path.join(_HERE, "libmvae_hip.so"))

P = c_void_p
I = c_int
L = c_longlong
F = c_float
D = c_double
Z = c_size_t

# name -> (restype, argtypes); mirrors include/medvae_hip.h one-to-one
SIGNATURES = {
    "mvae_last_error": (ctypes.c_char_p, []),
    "mvae_abi_version": (I, []),
    "mvae_set_math_mode": (I, [I]),
    "mvae_get_math_mode": (I, []),
    "mvae_set_dropout_salt": (I, [P]),
    "mvae_conv2d_nhwc": (I, [P, P, P, P, P, I, I, I, I, I, I, I, I, I, I, I, I, I, P]),
    "mvae_conv2d_direct32_nhwc": (I, [P, P, P, P, P, I, I, I, I, P]),
    "mvae_conv2d_ws_nhwc": (I, [P, P, P, P, P, I, I, I, I, I, I, I, I, I, I, I, I, I, P, Z, P]),
    "mvae_conv2d_split_workspace_bytes": (Z, [I, I, I, I, I, I, I]),
    "mvae_conv2d_gnstats_nhwc": (I, [P, P, P, P, P, I, I, I, I, I, I, I, I, I, I, I, I, I, P, P]),
    "mvae_conv2d_dgrad_gnbwd_nhwc": (I, [P, P, P, I, I, I, I, I, I, I, I, I, I, I, I, P, P, P, P, P, I, I, P, P]),
    "mvae_conv2d_wgrad_nhwc": (I, [P, P, P, P, F, I, I, I, I, I, I, I, I, I, I, I, I, I, P, Z, P]),
    "mvae_winograd_weight_transform": (I, [P, P, I, I, I, I, P]),
    "mvae_winograd_input_transform": (I, [P, P, I, I, I, I, I, I, P]),
    "mvae_winograd_input_transform_gn": (I, [P, P, P, I, P, I, I, I, I, I, P]),
    "mvae_group_norm_stats_nhwc": (I, [P, P, P, P, P, P, P, P, I, I, I, I, F, P, Z, P]),
    "mvae_group_norm_apply_nhwc": (I, [P, P, P, P, I, I, I, I, I, P]),
    "mvae_winograd_gemm": (I, [P, P, P, L, I, I, I, P]),
    "mvae_winograd_output_transform": (I, [P, P, P, P, P, I, I, I, I, I, P]),
    "mvae_winograd_output_gnbwd": (I, [P, P, P, P, P, P, P, I, I, P, I, I, I, I, I, P]),
    "mvae_winograd_dy_transform": (I, [P, P, I, I, I, I, I, I, P]),
    "mvae_winograd_dy_transforms": (I, [P, P, P, I, I, I, I, I, I, P]),
    "mvae_winograd_wgrad_gemm": (I, [P, P, P, L, I, I, I, P, Z, P]),
    "mvae_winograd_wgrad_output": (I, [P, P, F, I, I, I, P]),
    "mvae_winograd_upsample_weights": (I, [P, P, I, I, P]),
    "mvae_winograd_upsample_fold": (I, [P, P, F, I, I, P]),
    "mvae_winograd_output_transform_upsample": (I, [P, P, P, I, I, I, I, I, P]),
    "mvae_winograd_dy_transforms_upsample": (I, [P, P, P, I, I, I, I, I, P]),
    "mvae_conv2d_wgrad_workspace_bytes": (Z, [I, I, I, I, I, I, I]),
    "mvae_conv2d_wgrad_small_cout_nhwc": (I, [P, P, P, P, F, I, I, I, I, I, I, P, Z, P]),
    "mvae_conv2d_wgrad_small_cout_workspace_bytes": (Z, [I, I]),
    "mvae_conv2d_wgrad_direct_nhwc": (I, [P, P, P, P, F, I, I, I, I, I, I, P, Z, P]),
    "mvae_conv2d_wgrad_direct_workspace_bytes": (Z, [I, I, I, I, I]),
    "mvae_conv_weight_transpose": (I, [P, P, I, I, I, I, I, P]),
    "mvae_conv_weight_transpose_batched": (I, [P, I, I, P]),
    "mvae_conv_weight_upsample_dgrad": (I, [P, P, I, I, I, P]),
    "mvae_conv2d_dgrad_stride2_nhwc": (I, [P, P, P, I, I, I, I, I, I, I, I, I, I, I, I, P, Z, P]),
    "mvae_split_bf16": (I, [P, P, L, P]),
    "mvae_pack_bf16": (I, [P, P, L, P]),
    "mvae_pack_bf16_colsum": (I, [P, P, L, I, P, F, P, Z, P]),
    "mvae_split_planar": (I, [P, P, L, P]),
    "mvae_split_planar_colsum": (I, [P, P, L, I, P, F, P, Z, P]),
    "mvae_conv2d_upsample_nhwc": (I, [P, P, P, P, P, I, I, I, I, I, I, P]),
    "mvae_conv_weight_upsample_fwd": (I, [P, P, I, I, I, P]),
    "mvae_conv2d_wgrad_upsample_nhwc": (I, [P, P, P, P, F, I, I, I, I, I, P, Z, P]),
    "mvae_conv2d_wgrad_upsample_workspace_bytes": (Z, [I, I, I, I, I]),
    "mvae_bias_grad": (I, [P, L, I, L, P, F, P, Z, P]),
    "mvae_bias_grad_workspace_bytes": (Z, [L, I]),
    "mvae_gemm_strided_batched": (I, [I, I, I, I, I, F, P, L, L, P, L, L, F, P, L, L, I, P, P, L, L, P, Z, P]),
    "mvae_gemm_workspace_bytes": (Z, [I, I, I, I]),
    "mvae_softmax_rows": (I, [P, P, L, I, P]),
    "mvae_softmax_rows_bwd": (I, [P, P, P, L, I, P]),
    "mvae_attention_small_fwd": (I, [P, P, P, P, P, I, I, I, F, P]),
    "mvae_attention_small_bwd": (I, [P, P, P, P, P, P, P, P, I, I, I, F, P]),
    "mvae_attention_tile_fwd": (I, [P, P, P, P, P, I, I, I, F, P]),
    "mvae_attention_tile_bwd": (I, [P, P, P, P, P, P, I, I, I, F, P]),
    "mvae_group_norm_fwd_nhwc": (I, [P, P, P, P, P, P, I, I, I, I, F, I, F, c_uint64, I, P, Z, P]),
    "mvae_group_norm_fwd_part_nhwc": (I, [P, P, P, P, P, P, P, I, I, I, I, F, I, F, c_uint64, I, P, Z, P]),
    "mvae_group_norm_bwd_nhwc": (I, [P, P, P, P, P, P, P, P, P, P, I, I, I, I, I, F, c_uint64, P, Z, P]),
    "mvae_group_norm_bwd_part_nhwc": (I, [P, P, P, P, P, P, P, P, P, P, P, I, I, I, I, I, P, Z, P]),
    "mvae_group_norm_bwd_part_split_nhwc": (I, [P, P, P, P, P, P, P, P, P, P, P, I, I, I, I, I, P, Z, P, P, F, P, Z,
                                               P]),
    "mvae_group_norm_bwd_streaming": (I, [I, I, I, I, I]),
    "mvae_group_norm_workspace_bytes": (Z, [I, I, I]),
    "mvae_group_norm_bwd_pack_nhwc": (I, [P, P, P, P, P, P, P, P, P, P, I, I, I, I, I, F, c_uint64, P, Z, P, P, F, P, Z,
                                          P]),
    "mvae_group_norm_bwd_split_nhwc": (I, [P, P, P, P, P, P, P, P, P, P, I, I, I, I, I, F, c_uint64, P, Z, P, P, F, P, Z,
                                          P]),
    "mvae_group_norm_bwd_colsum_nhwc": (I, [P, P, P, P, P, P, P, P, P, P, I, I, I, I, I, F, c_uint64, P, Z, P, F, P, Z,
                                           P]),
    "mvae_group_norm_colsum_workspace_bytes": (Z, [I, I, I]),
    "mvae_set_group_norm_path": (I, [I]),
    "mvae_reparam_fwd": (I, [P, P, L, P, P, L, I, P]),
    "mvae_reparam_bwd": (I, [P, P, P, L, P, L, I, P]),
    "mvae_loss_reduce": (I, [I, P, P, L, L, I, D, P, P, Z, P]),
    "mvae_reduce_workspace_bytes": (Z, []),
    "mvae_kl_bwd": (I, [P, P, L, P, D, P, P, L, I, P]),
    "mvae_latent_prep_fwd": (I, [P, P, L, P, P, P, P, P, L, I, P]),
    "mvae_latent_prep_bwd": (I, [P, P, L, P, P, P, P, P, P, P, L, L, I, P]),
    "mvae_loss_combine4_fwd": (I, [P, P, P, P, F, F, F, F, I, F, P, P, P, P, P, P, P]),
    "mvae_loss_combine4_bwd": (I, [P, F, F, F, F, I, P, P, P, P, P, P, P]),
    "mvae_recon_bwd": (I, [I, P, P, P, D, P, L, P]),
    "mvae_multi_tensor_adam": (I, [P, P, P, P, P, P, P, I, P, I, P, P, F, F, I, F, F, F, F, F, I, P, Z, P, P]),
    "mvae_multi_tensor_adam_workspace_bytes": (Z, [I, I]),
    "mvae_lpips_scale": (I, [P, P, L, I, F, F, P, P, P]),
    "mvae_lpips_scale_bwd": (I, [P, P, L, I, F, P, P]),
    "mvae_relu_fwd": (I, [P, P, L, P]),
    "mvae_relu_bwd": (I, [P, P, P, L, P]),
    "mvae_maxpool_fwd": (I, [P, P, P, I, I, I, I, I, I, P]),
    "mvae_maxpool_bwd": (I, [P, P, P, I, I, I, I, I, I, P]),
    "mvae_lpips_dist": (I, [P, P, P, P, I, I, I, F, P]),
    "mvae_lpips_dist_bwd": (I, [P, P, P, P, P, P, I, I, I, P]),
    "mvae_ssim": (I, [P, P, I, I, I, I, F, P, P]),
    "mvae_kl_stats": (I, [P, P, L, L, I, P, P, Z, P]),
    "mvae_kl_stats_workspace_bytes": (Z, [L]),
    "mvae_decode_batch": (I, [P, P, P, P, P, P, P, P, I, I, I, I, I, P, P, P, P, P, Z, P]),
    "mvae_decode_batch_workspace_bytes": (Z, [I, I]),
    "mvae_adv_bwd": (I, [I, P, P, D, P, L, P]),
    "mvae_batch_norm_fwd_nhwc": (I, [P, P, P, P, P, P, P, P, L, I, F, F, I, F, P, Z, P]),
    "mvae_batch_norm_bwd_nhwc": (I, [P, P, P, P, P, P, P, P, P, L, I, F, P, Z, P]),
    "mvae_batch_norm_workspace_bytes": (Z, [L, I]),
    "mvae_leaky_relu_fwd": (I, [P, P, F, L, P]),
    "mvae_leaky_relu_bwd": (I, [P, P, P, F, L, P]),
    "mvae_modality_heads_fwd": (I, [P, P, I, I, I, I, I, P, I, P, P]),
    "mvae_modality_heads_bwd": (I, [P, P, I, I, I, I, I, P, I, P, P, P, P, Z, P]),
    "mvae_modality_heads_workspace_bytes": (Z, [I, I]),
    "mvae_modality_route_in_fwd": (I, [P, I, P, I, I, I, I, P, P, P]),
    "mvae_modality_route_in_bwd": (I, [P, I, P, I, I, I, I, P, P, P, P, Z, P]),
    "mvae_modality_route_in_workspace_bytes": (Z, [I, I]),
    "mvae_condition_concat_fwd": (I, [P, P, P, P, P, P, I, I, I, I, I, P]),
    "mvae_condition_concat_bwd": (I, [P, P, P, P, P, P, I, I, I, I, I, P]),
    "mvae_latent_aux_fwd": (I, [P, P, I, I, I, I, I, I, F, P, P, Z, P]),
    "mvae_latent_aux_bwd": (I, [P, P, I, I, I, I, I, I, F, P, P, P, P, P, Z, P]),
    "mvae_latent_aux_workspace_bytes": (Z, [I, I]),
}


class HipLibraryError(RuntimeError):
    pass


_lib = None


def load():
    """Load libmvae_hip.so (raises HipLibraryError if it is missing: there is no CPU fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise HipLibraryError(
            f"{LIB_PATH} not found: build it with `make` (or __graft_entry__.build()); "
            "the MI355X path has no CPU fallback")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    _bind_fast(lib)
    return lib


# Low-overhead call path (csrc/pyfast.c, built in-tree next to the library): the same entry points of the same
# library, called through one SysV trampoline instead of ctypes' per-call argument conversion (~0.3 vs ~3-5 us).
# Entry points it cannot take (and every call when the module is not built) stay on ctypes.
_CODE = {P: "P", I: "I", L: "L", F: "F", D: "D", Z: "Z"}
_CODE.setdefault(c_uint64, "U")  # (c_uint64 is c_size_t on LP64: one unsigned 64-bit class either way)
_FAST = {}
_fast_mod = None


def _bind_fast(lib):
    global _fast_mod
    if os.environ.get("MVAE_NO_FASTCALL") is not None:
        return
    try:
        from . import _mvae_fast as fm
    except ImportError:
        return
    for name, (res, args) in SIGNATURES.items():
        if res not in (I, Z) or any(t not in _CODE for t in args):
            continue
        idx = fm.bind(ctypes.cast(getattr(lib, name), c_void_p).value, _CODE[res] + "".join(_CODE[t] for t in args))
        if idx is not None:
            _FAST[name] = idx
    _fast_mod = fm


def call(name, *args):
    """Invoke an int-returning entry point and raise on a non-zero status."""
    lib = load()
    idx = _FAST.get(name)
    if idx is None:
        rc = getattr(lib, name)(*args)
    else:
        try:
            rc = _fast_mod.call(idx, *args)
        except TypeError:  # a ctypes object argument (pointer arrays): converted before any call, so retry there
            rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.mvae_last_error().decode(errors="replace")
        raise RuntimeError(f"{name} failed (status {rc}): {msg}")
    return rc


def query(name, *args):
    lib = load()
    idx = _FAST.get(name)
    return _fast_mod.call(idx, *args) if idx is not None else getattr(lib, name)(*args)
