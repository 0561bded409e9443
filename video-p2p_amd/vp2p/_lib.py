"""ctypes binding of libvp2p_hip.so (include/vp2p.h).

The C ABI takes plain device pointers, element strides and a hipStream_t; this module only
mirrors the structs and resolves the symbols.  ``load()`` raises if the library is missing or
stale: there is no CPU or PyTorch fallback for any op in this package.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_float, c_int32, c_int64, c_void_p

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("VP2P_LIB", os.path.join(os.path.dirname(_HERE), "lib", "libvp2p_hip.so"))

ABI_VERSION = 16
F32, BF16 = 0, 1
EDIT_NONE, EDIT_REPLACE, EDIT_REFINE = 0, 1, 2
CONV_EPI_NONE, CONV_EPI_GEGLU = 0, 1
STATUS = {0: "OK", -1: "VP2P_E_ARG", -2: "VP2P_E_DTYPE", -3: "VP2P_E_HEAD_DIM", -4: "VP2P_E_SHAPE",
          -5: "VP2P_E_LAUNCH"}

EXPORTS = ("vp2p_frame_attn_fwd", "vp2p_cross_kv_workspace_bytes", "vp2p_cross_kv_prep",
           "vp2p_cross_attn_p2p_fwd", "vp2p_temporal_attn_p2p_fwd", "vp2p_step_fused",
           "vp2p_abi_version", "vp2p_supported_head_dims",
           "vp2p_group_norm_parts", "vp2p_group_norm_stats", "vp2p_group_norm_apply", "vp2p_group_norm_fwd",
           "vp2p_layer_norm_fwd", "vp2p_geglu_fwd",
           "vp2p_frame_attn_bwd_workspace_bytes", "vp2p_frame_attn_bwd", "vp2p_temporal_attn_bwd",
           "vp2p_group_norm_bwd_reduce", "vp2p_group_norm_bwd_apply", "vp2p_layer_norm_bwd", "vp2p_geglu_bwd",
           "vp2p_nulltext_loss", "vp2p_nulltext_loss_partials", "vp2p_conv2d_supported", "vp2p_conv2d_fwd",
           "vp2p_add_layer_norm_fwd", "vp2p_conv2d_workspace_bytes", "vp2p_group_norm_finalize",
           "vp2p_group_norm_apply_stats", "vp2p_group_norm_merge", "vp2p_group_norm_finalize_merged",
           "vp2p_group_norm_finalize_parts", "vp2p_group_norm_merge_parts", "vp2p_conv2d_gn_parts",
           "vp2p_group_norm_apply_parts", "vp2p_conv2d_plan")


class GroupNormArgs(ctypes.Structure):
    _fields_ = [("x", c_void_p), ("add", c_void_p), ("y", c_void_p), ("weight", c_void_p), ("bias", c_void_p),
                ("partials", c_void_p), ("batch", c_int32), ("frames", c_int32), ("rows", c_int32),
                ("channels", c_int32), ("groups", c_int32), ("eps", c_float), ("silu", c_int32),
                ("dtype", c_int32), ("x2", c_void_p), ("channels2", c_int32)]


class ConvArgs(ctypes.Structure):
    _fields_ = [("x", c_void_p), ("w", c_void_p), ("bias", c_void_p), ("residual", c_void_p), ("y", c_void_p),
                ("batch", c_int32), ("in_h", c_int32), ("in_w", c_int32), ("cin", c_int32),
                ("cout", c_int32), ("out_h", c_int32), ("out_w", c_int32),
                ("kernel", c_int32), ("stride", c_int32), ("pad", c_int32), ("dtype", c_int32),
                ("epilogue", c_int32), ("workspace", c_void_p), ("ksplit", c_int32),
                ("upsample", c_int32), ("x2", c_void_p), ("cin2", c_int32), ("alpha", c_float),
                ("img_add", c_void_p), ("gn_partials", c_void_p), ("gn_groups", c_int32), ("gn_rows", c_int32)]


class LayerNormArgs(ctypes.Structure):
    _fields_ = [("x", c_void_p), ("y", c_void_p), ("weight", c_void_p), ("bias", c_void_p),
                ("rows", c_int64), ("channels", c_int32), ("eps", c_float), ("dtype", c_int32)]


class FrameAttnArgs(ctypes.Structure):
    _fields_ = [("q", c_void_p), ("k", c_void_p), ("v", c_void_p), ("o", c_void_p),
                ("q_sb", c_int64), ("q_sf", c_int64), ("q_sn", c_int64),
                ("k_sb", c_int64), ("k_sn", c_int64),
                ("v_sb", c_int64), ("v_sn", c_int64),
                ("o_sb", c_int64), ("o_sf", c_int64), ("o_sn", c_int64),
                ("batch", c_int32), ("frames", c_int32), ("tokens_q", c_int32), ("tokens_kv", c_int32),
                ("heads", c_int32), ("head_dim", c_int32), ("scale", c_float), ("dtype", c_int32),
                ("lse", c_void_p), ("q_prescaled", c_int32)]


class FrameAttnBwdArgs(ctypes.Structure):
    _fields_ = [("q", c_void_p), ("k", c_void_p), ("v", c_void_p), ("o", c_void_p), ("dout", c_void_p),
                ("lse", c_void_p), ("dq", c_void_p), ("dk", c_void_p), ("dv", c_void_p), ("workspace", c_void_p),
                ("q_sb", c_int64), ("q_sf", c_int64), ("q_sn", c_int64), ("kv_sb", c_int64), ("kv_sn", c_int64),
                ("batch", c_int32), ("frames", c_int32), ("tokens_q", c_int32), ("tokens_kv", c_int32),
                ("heads", c_int32), ("head_dim", c_int32), ("scale", c_float), ("dtype", c_int32)]


class TemporalAttnBwdArgs(ctypes.Structure):
    _fields_ = ([("q", c_void_p), ("k", c_void_p), ("v", c_void_p), ("dout", c_void_p),
                 ("dq", c_void_p), ("dk", c_void_p), ("dv", c_void_p)]
                + [(f"{t}_s{x}", c_int64) for t in ("q", "k", "v", "do", "dq", "dk", "dv") for x in "bfn"]
                + [("batch", c_int32), ("frames", c_int32), ("tokens", c_int32), ("heads", c_int32),
                   ("head_dim", c_int32), ("scale", c_float), ("dtype", c_int32)])


class CrossAttnArgs(ctypes.Structure):
    _fields_ = [("q", c_void_p), ("kv_ws", c_void_p), ("o", c_void_p),
                ("q_sb", c_int64), ("q_sf", c_int64), ("q_sn", c_int64),
                ("o_sb", c_int64), ("o_sf", c_int64), ("o_sn", c_int64),
                ("batch", c_int32), ("frames", c_int32), ("tokens_q", c_int32), ("tokens_kv", c_int32),
                ("heads", c_int32), ("head_dim", c_int32), ("scale", c_float), ("dtype", c_int32),
                ("prompts", c_int32), ("edit_mode", c_int32), ("reweight", c_int32),
                ("alpha_words", c_void_p), ("map_ptr", c_void_p), ("map_idx", c_void_p),
                ("map_val", c_void_p), ("refine_alpha", c_void_p), ("equalizer", c_void_p),
                ("lb_acc", c_void_p), ("lb_word_alpha", c_void_p), ("probs_out", c_void_p),
                ("lb_ws", c_void_p), ("lb_sets", c_int32), ("cond_only", c_int32)]


class TemporalAttnArgs(ctypes.Structure):
    _fields_ = [("q", c_void_p), ("k", c_void_p), ("v", c_void_p), ("o", c_void_p),
                ("q_sb", c_int64), ("q_sf", c_int64), ("q_sn", c_int64),
                ("k_sb", c_int64), ("k_sf", c_int64), ("k_sn", c_int64),
                ("v_sb", c_int64), ("v_sf", c_int64), ("v_sn", c_int64),
                ("o_sb", c_int64), ("o_sf", c_int64), ("o_sn", c_int64),
                ("batch", c_int32), ("frames", c_int32), ("tokens", c_int32), ("heads", c_int32),
                ("head_dim", c_int32), ("scale", c_float), ("dtype", c_int32),
                ("prompts", c_int32), ("self_replace", c_int32), ("probs_out", c_void_p),
                ("cond_only", c_int32)]


class StepArgs(ctypes.Structure):
    _fields_ = [("noise", c_void_p), ("noise_dtype", c_int32), ("latents", c_void_p), ("out", c_void_p),
                ("prompts", c_int32), ("channels", c_int32), ("frames", c_int32), ("height", c_int32),
                ("width", c_int32), ("cfg", c_int32), ("fast", c_int32), ("guidance", c_float),
                ("c1", c_float), ("c2", c_float), ("c3", c_float), ("c4", c_float),
                ("lb_acc", c_void_p), ("lb_h", c_int32), ("lb_w", c_int32), ("lb_count", c_float),
                ("lb_th", c_float), ("lb_sub", c_void_p), ("lb_sub_th", c_float), ("mask_out", c_void_p)]


class NullTextLossArgs(ctypes.Structure):
    _fields_ = [("noise_uncond", c_void_p), ("noise_cond", c_void_p), ("noise_dtype", c_int32),
                ("latents", c_void_p), ("latents_prev", c_void_p), ("grad_uncond", c_void_p),
                ("partials", c_void_p), ("loss", c_void_p), ("n", c_int64),
                ("guidance", c_float), ("c1", c_float), ("c2", c_float), ("c3", c_float), ("c4", c_float)]


class Vp2pError(RuntimeError):
    pass


_LIB = None


def load(path: str = None):
    """Load and type the library once.  Raises ``Vp2pError`` if it is absent or mismatched."""
    global _LIB
    if _LIB is not None and path is None:
        return _LIB
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise Vp2pError(f"libvp2p_hip.so not found at {p}: build it with `make -C video-p2p_amd` "
                        "(there is no CPU fallback)")
    try:  # share torch's HIP runtime (same SONAME) when torch is already loaded
        import torch  # noqa: F401
    except Exception:
        pass
    lib = ctypes.CDLL(p, mode=ctypes.RTLD_GLOBAL)
    lib.vp2p_frame_attn_fwd.argtypes = [POINTER(FrameAttnArgs), c_void_p]
    lib.vp2p_cross_kv_workspace_bytes.argtypes = [c_int32] * 5
    lib.vp2p_cross_kv_workspace_bytes.restype = c_int64
    lib.vp2p_cross_kv_prep.argtypes = [c_void_p, c_void_p, c_int64, c_int64, c_int64, c_int64,
                                       c_int32, c_int32, c_int32, c_int32, c_int32, c_void_p, c_void_p]
    lib.vp2p_cross_attn_p2p_fwd.argtypes = [POINTER(CrossAttnArgs), c_void_p]
    lib.vp2p_temporal_attn_p2p_fwd.argtypes = [POINTER(TemporalAttnArgs), c_void_p]
    lib.vp2p_step_fused.argtypes = [POINTER(StepArgs), c_void_p]
    lib.vp2p_supported_head_dims.argtypes = [POINTER(c_int32), c_int32]
    gn = POINTER(GroupNormArgs)
    lib.vp2p_group_norm_parts.argtypes = [gn]
    lib.vp2p_group_norm_stats.argtypes = [gn, c_void_p]
    lib.vp2p_group_norm_apply.argtypes = [gn, c_void_p, c_int32, c_void_p]
    lib.vp2p_group_norm_fwd.argtypes = [gn, c_void_p]
    lib.vp2p_group_norm_finalize.argtypes = [gn, c_void_p, c_int32, c_void_p, c_void_p]
    lib.vp2p_group_norm_apply_stats.argtypes = [gn, c_void_p, c_void_p]
    lib.vp2p_group_norm_merge.argtypes = [gn, c_void_p, c_void_p, c_void_p]
    lib.vp2p_group_norm_finalize_merged.argtypes = [gn, c_void_p, c_int32, c_void_p, c_void_p]
    lib.vp2p_layer_norm_fwd.argtypes = [POINTER(LayerNormArgs), c_void_p]
    lib.vp2p_geglu_fwd.argtypes = [c_void_p, c_void_p, c_int64, c_int32, c_int32, c_void_p]
    lib.vp2p_frame_attn_bwd_workspace_bytes.argtypes = [POINTER(FrameAttnBwdArgs)]
    lib.vp2p_frame_attn_bwd_workspace_bytes.restype = c_int64
    lib.vp2p_frame_attn_bwd.argtypes = [POINTER(FrameAttnBwdArgs), c_void_p]
    lib.vp2p_temporal_attn_bwd.argtypes = [POINTER(TemporalAttnBwdArgs), c_void_p]
    lib.vp2p_group_norm_bwd_reduce.argtypes = [gn, c_void_p, c_int32, c_void_p, c_void_p, c_void_p]
    lib.vp2p_group_norm_bwd_apply.argtypes = [gn, c_void_p, c_int32, c_void_p, c_void_p, c_int32, c_void_p,
                                              c_void_p]
    lib.vp2p_layer_norm_bwd.argtypes = [POINTER(LayerNormArgs), c_void_p, c_void_p, c_void_p]
    lib.vp2p_geglu_bwd.argtypes = [c_void_p, c_void_p, c_void_p, c_int64, c_int32, c_int32, c_void_p]
    lib.vp2p_nulltext_loss.argtypes = [POINTER(NullTextLossArgs), c_void_p]
    lib.vp2p_nulltext_loss_partials.argtypes = []
    lib.vp2p_conv2d_supported.argtypes = [POINTER(ConvArgs)]
    lib.vp2p_conv2d_fwd.argtypes = [POINTER(ConvArgs), c_void_p]
    lib.vp2p_conv2d_workspace_bytes.argtypes = [POINTER(ConvArgs)]
    lib.vp2p_conv2d_gn_parts.argtypes = [POINTER(ConvArgs)]
    lib.vp2p_conv2d_plan.argtypes = [POINTER(ConvArgs), POINTER(c_int32), POINTER(c_int32)]
    lib.vp2p_group_norm_finalize_parts.argtypes = [gn, c_void_p, c_int32, c_void_p, c_void_p]
    lib.vp2p_group_norm_merge_parts.argtypes = [gn, c_void_p, c_int32, c_void_p, c_void_p]
    lib.vp2p_group_norm_apply_parts.argtypes = [gn, c_void_p, c_int32, c_void_p]
    lib.vp2p_conv2d_workspace_bytes.restype = c_int64
    lib.vp2p_add_layer_norm_fwd.argtypes = [POINTER(LayerNormArgs), c_void_p, c_void_p, c_void_p]
    for name in ("vp2p_frame_attn_fwd", "vp2p_cross_kv_prep", "vp2p_cross_attn_p2p_fwd",
                 "vp2p_temporal_attn_p2p_fwd", "vp2p_step_fused", "vp2p_abi_version",
                 "vp2p_supported_head_dims", "vp2p_group_norm_parts", "vp2p_group_norm_stats",
                 "vp2p_group_norm_apply", "vp2p_group_norm_fwd", "vp2p_layer_norm_fwd", "vp2p_geglu_fwd",
                 "vp2p_frame_attn_bwd", "vp2p_temporal_attn_bwd", "vp2p_group_norm_bwd_reduce",
                 "vp2p_group_norm_bwd_apply", "vp2p_layer_norm_bwd", "vp2p_geglu_bwd", "vp2p_nulltext_loss",
                 "vp2p_nulltext_loss_partials", "vp2p_conv2d_supported", "vp2p_conv2d_fwd",
                 "vp2p_add_layer_norm_fwd", "vp2p_group_norm_finalize", "vp2p_group_norm_apply_stats",
                 "vp2p_group_norm_merge", "vp2p_group_norm_finalize_merged", "vp2p_group_norm_finalize_parts",
                 "vp2p_group_norm_merge_parts", "vp2p_conv2d_gn_parts", "vp2p_group_norm_apply_parts",
                 "vp2p_conv2d_plan"):
        getattr(lib, name).restype = c_int32
    if lib.vp2p_abi_version() != ABI_VERSION:
        raise Vp2pError(f"{p}: ABI version {lib.vp2p_abi_version()} != {ABI_VERSION}; rebuild")
    if path is None:
        _LIB = lib
    return lib


def check(rc: int, what: str):
    if rc != 0:
        raise Vp2pError(f"{what} failed: {STATUS.get(rc, rc)}")


def supported_head_dims():
    lib = load()
    buf = (c_int32 * 16)()
    n = lib.vp2p_supported_head_dims(buf, 16)
    return [buf[i] for i in range(n)]
