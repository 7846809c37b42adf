"""ctypes binding of libsfm_amd.so (the C ABI declared in include/sfm_amd.h).

The library is built in-tree (``make -C self-supervise-sfm_amd/csrc``) and loaded
from this package directory.  torch is imported first so that the HIP runtime
(``libamdhip64.so.7``) the library depends on resolves to the one torch already
loaded — one runtime, one set of streams.  There is no fallback: if the library is
missing, every op raises.
"""

from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must load the HIP runtime before the library)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SFM_AMD_LIB") or os.path.join(_HERE, "libsfm_amd.so")  # override: tuning builds

SR_F32, SR_BF16 = 0, 1
SR_EPI_BIAS, SR_EPI_BIAS_GELU, SR_EPI_BIAS_RESID, SR_EPI_QKV, SR_EPI_PATCH = 0, 1, 2, 3, 4
SR_EPI_F32, SR_EPI_GELU_BWD = 5, 6
SR_MASK_NONE, SR_MASK_CAMERA, SR_MASK_DENSE, SR_MASK_ADD = 0, 1, 2, 3
SR_ATTN_MERGE_MAX_PARTS = 16

_vp = ctypes.c_void_p
_i64 = ctypes.c_int64
_i32 = ctypes.c_int
_f32 = ctypes.c_float


class GemmEpi(ctypes.Structure):
    _fields_ = [
        ("bias", _vp), ("gamma", _vp),
        ("qn_w", _vp), ("qn_b", _vp), ("kn_w", _vp), ("kn_b", _vp), ("qk_eps", _f32),
        ("rope_cos", _vp), ("rope_sin", _vp), ("rope_npos", _i32),
        ("col_offset", _i32), ("head_dim", _i32), ("embed_dim", _i32),
        ("pos_yx", _vp), ("pos_rowmap", _vp), ("pos_row_base", _i64),
        ("tokens_per_frame", _i32), ("patch_start", _i32), ("grid_w", _i32),
        ("seg_rows", _i32), ("seg_stride", _i32), ("seg_offset", _i32), ("row_add", _vp),
        ("aux", _vp), ("ld_aux", _i64),
        ("q_scale", _f32), ("q_cols", _i32), ("colsum", _vp),
    ]


class GemmProblem(ctypes.Structure):
    _fields_ = [
        ("A", _vp), ("lda", _i64), ("W", _vp), ("ldw", _i64), ("out", _vp), ("ldo", _i64),
        ("M", _i32), ("N", _i32), ("K", _i32), ("ep", GemmEpi),
    ]


class WgradProblem(ctypes.Structure):
    _fields_ = [
        ("A", _vp), ("lda", _i64), ("B", _vp), ("ldb", _i64), ("dW", _vp), ("lddw", _i64),
        ("M", _i32), ("N", _i32), ("K", _i32), ("accumulate", _i32),
        ("rowscale", _vp), ("wdot", _vp), ("ldwd", _i64), ("rowdot", _vp), ("splits", _i32), ("workspace", _vp),
    ]


class AttnDesc(ctypes.Structure):
    _fields_ = [
        ("q", _vp), ("ldq", _i64),
        ("k0", _vp), ("v0", _vp), ("ldk0", _i64), ("ldv0", _i64),
        ("k1", _vp), ("v1", _vp), ("ldk1", _i64), ("ldv1", _i64),
        ("o", _vp), ("ldo", _i64),
        ("batch", _i32), ("heads", _i32), ("head_dim", _i32),
        ("lq", _i32), ("q_bstride", _i64),
        ("l0", _i32), ("k0_bstride", _i64),
        ("l1", _i32), ("k1_bstride", _i64),
        ("mask_mode", _i32), ("n_anchor", _i32),
        ("scale", _f32),
        ("lse", _vp),
        ("key_bound", _vp),
        ("key_norm_max", _f32),
        ("o_bstride", _i64),
        ("mask", _vp), ("mask_bstride", _i64), ("mask_hstride", _i64), ("mask_ld", _i64),
        ("tail_rows_readable", _i32),
        ("merge_o", _vp), ("ld_merge_o", _i64), ("merge_lse", _vp), ("merge_rows", _i64),
        ("sweep_stats", _vp),
        ("key_box", _vp),
        ("value_box", _vp),
        ("key_norm2", _vp),
        ("q_scaled", _i32),
    ]


class WeightItem(ctypes.Structure):
    """sr_weight_item (include/sfm_amd.h)."""
    _fields_ = [
        ("src", _vp),
        ("lds", _i64),
        ("rows", _i32),
        ("cols", _i32),
        ("rowscale", _vp),
        ("cast", _vp),
        ("ldc", _i64),
        ("trans", _vp),
        ("ldt", _i64),
    ]


SR_WEIGHT_REFRESH_MAX = 4


class AttnBwdDesc(ctypes.Structure):
    _fields_ = [
        ("f", AttnDesc),
        ("dout", _vp), ("lddo", _i64),
        ("delta", _vp),
        ("dq", _vp), ("lddq", _i64),
        ("dk0", _vp), ("dv0", _vp), ("lddk0", _i64), ("lddv0", _i64),
        ("dk1", _vp), ("dv1", _vp), ("lddk1", _i64), ("lddv1", _i64),
    ]


class ImcLossDesc(ctypes.Structure):
    _fields_ = [
        ("enc", _vp), ("n_views", _i32), ("H", _i32), ("W", _i32), ("kp2k", _vp), ("shared_focal", _i32),
        ("n_pairs", _i32), ("n_points", _i32), ("src_idx", _vp), ("dst_idx", _vp), ("src_coords", _vp),
        ("dst_coords", _vp), ("src_depth", _vp), ("dst_depth", _vp), ("node_src", _vp), ("node_dst", _vp),
        ("n_nodes", _i32), ("min_val", _f32), ("max_val", _f32), ("num_bins", _i32), ("smooth_w", _vp),
        ("smooth_radius", _i32), ("grad_scale", _f32), ("loss", _vp), ("d_enc", _vp), ("workspace", _vp),
    ]


# name -> (restype, argtypes)
_PROTOS = {
    "sr_last_error": (ctypes.c_char_p, []),
    "sr_version": (_i32, []),
    "sr_last_kernel": (ctypes.c_char_p, []),
    "sr_set_tuning": (_i32, [_i32, _i32]),
    "sr_get_tuning": (_i32, [_i32]),
    "sr_tuning_name": (ctypes.c_char_p, [_i32]),
    "sr_gemm": (_i32, [_vp, _i32, _i32, _vp, _i64, _vp, _i64, _vp, _i64, _i32, _i32, _i32, ctypes.POINTER(GemmEpi)]),
    "sr_gemm_splitk": (_i32, [_vp, _i32, _i32, _vp, _i64, _vp, _i64, _vp, _i64, _i32, _i32, _i32, _i32, _vp,
                              ctypes.POINTER(GemmEpi)]),
    "sr_attention": (_i32, [_vp, _i32, ctypes.POINTER(AttnDesc)]),
    "sr_attention_pair": (_i32, [_vp, _i32, ctypes.POINTER(AttnDesc), ctypes.POINTER(AttnDesc)]),
    "sr_attention_pair_vt": (_i32, [_vp, _i32, ctypes.POINTER(AttnDesc), ctypes.POINTER(AttnDesc), _vp, _vp]),
    "sr_vt_tiles": (_i32, [_vp, _vp, _i64, _i32, _i32, _vp]),
    "sr_gemm_group": (_i32, [_vp, _i32, _i32, _i32, ctypes.POINTER(GemmProblem)]),
    "sr_attention_bound_floats": (_i32, [ctypes.POINTER(AttnDesc)]),
    "sr_attn_merge_n": (_i32, [_vp, _i32, _i32, _i32, _i32, _i32, _vp, _i64, _i64, _vp, _vp, _vp, _i64, _vp]),
    "sr_attn_merge": (_i32, [_vp, _i32, _i32, _i32, _i32, _vp, _i64, _vp, _vp, _i64, _vp, _vp, _i64, _vp]),
    "sr_quant_fp8": (_i32, [_vp, _vp, _i64, _i32, _i32, _f32, _vp, _i64, _vp, _vp]),
    "sr_attention_qk8": (_i32, [_vp, ctypes.POINTER(AttnDesc), _vp, _i64, _vp, _i64, _vp]),
    "sr_quant_fp8_vt": (_i32, [_vp, _vp, _i64, _i32, _i32, _vp, _vp, _vp]),
    "sr_attention_qkv8": (_i32, [_vp, ctypes.POINTER(AttnDesc), _vp, _i64, _vp, _i64, _vp, _vp]),
    "sr_attention_bwd": (_i32, [_vp, ctypes.POINTER(AttnBwdDesc)]),
    "sr_attention_bwd_f32": (_i32, [_vp, ctypes.POINTER(AttnBwdDesc)]),
    "sr_im2col3x3_f32": (_i32, [_vp, _vp, _i32, _i32, _i32, _i32, _i32, _i32, _vp]),
    "sr_conv3x3_f32": (_i32, [_vp, _vp, _i32, _i32, _i32, _i32, _i32, _i32, _vp, _i32, _i32,
                              ctypes.POINTER(GemmEpi), _vp, _i64, _vp]),
    "sr_convt_scatter_f32": (_i32, [_vp, _vp, _i32, _i32, _i32, _i32, _i32, _vp, _vp]),
    "sr_resize_bilinear_f32": (_i32, [_vp, _vp, _i32, _i32, _i32, _i32, _i32, _i32, _vp, _vp]),
    "sr_add_f32": (_i32, [_vp, _vp, _vp, _i64]),
    "sr_relu_f32": (_i32, [_vp, _vp, _i64]),
    "sr_dpt_pos_embed_f32": (_i32, [_vp, _vp, _i32, _i32, _i32, _i32, _f32, _f32]),
    "sr_dpt_head_out_f32": (_i32, [_vp, _vp, _i64, _i64, _i32, _vp, _vp, _i32, _i32, _i32, _vp, _vp]),
    "sr_unproject_depth_f32": (_i32, [_vp, _vp, _vp, _vp, _i32, _i32, _i32, _vp]),
    "sr_pil_resample_h": (_i32, [_vp, _i32, _vp, _i32, _i32, _i32, _i32, _vp, _vp, _i32, _i32, _vp]),
    "sr_pil_resample_v_f32": (_i32, [_vp, _i32, _vp, _i32, _i32, _i32, _i32, _vp, _vp, _i32, _i32, _f32, _vp,
                                     _i64, _i64, _i64]),
    "sr_layernorm": (_i32, [_vp, _i32, _vp, _i64, _vp, _vp, _vp, _f32, _vp, _i64, _i32, _i32]),
    "sr_layernorm_copy": (_i32, [_vp, _i32, _vp, _i64, _vp, _vp, _f32, _vp, _i64, _vp, _i64, _i32, _i32]),
    "sr_residual_layernorm": (_i32, [_vp, _i32, _vp, _i64, _vp, _i64, _vp, _vp, _vp, _f32, _vp, _i64, _i32, _i32]),
    "sr_im2col_normalize": (_i32, [_vp, _i32, _vp, _i32, _i32, _i32, _i32, ctypes.POINTER(_f32),
                                   ctypes.POINTER(_f32), _vp, _i32]),
    "sr_set_special_tokens": (_i32, [_vp, _vp, _i64, _i32, _i32, _i32, _vp, _vp, _i32]),
    "sr_copy_rows_f32": (_i32, [_vp, _vp, _i64, _vp, _i64, _vp, _i32, _i32]),
    "sr_mul_cols": (_i32, [_vp, _i32, _vp, _i64, _vp, _vp, _i64, _i32, _i32]),
    "sr_linear_small_f32": (_i32, [_vp, _vp, _i64, _vp, _vp, _vp, _i64, _i32, _i32, _i32, _i32]),
    "sr_silu_f32": (_i32, [_vp, _vp, _vp, _i64]),
    "sr_adaln_modulate_f32": (_i32, [_vp, _vp, _vp, _vp, _vp, _i32, _i32]),
    "sr_pose_update_f32": (_i32, [_vp, _vp, _vp, _i64, _vp, _i32, _i32]),
    "sr_pose_decode_f32": (_i32, [_vp, _vp, _i64, _i32, _i32, _i32, _vp, _vp]),
    # training step
    "sr_gemm_wgrad_pair": (_i32, [_vp, ctypes.POINTER(WgradProblem)]),
    "sr_gemm_wgrad": (_i32, [_vp, _vp, _i64, _vp, _i64, _vp, _i64, _i32, _i32, _i32, _i32, _vp, _vp, _i64, _vp,
                             _i32, _vp]),
    "sr_colsum": (_i32, [_vp, _i32, _vp, _i64, _i32, _i32, _vp, _i32, _f32, _vp, _i64]),
    "sr_colsum_workspace_floats": (_i64, [_i32, _i32]),
    "sr_layernorm_bwd": (_i32, [_vp, _i32, _vp, _i64, _vp, _vp, _i64, _vp, _f32, _vp, _i64, _vp, _i64, _vp, _vp,
                                _i32, _i32, _vp, _vp]),
    "sr_qk_bwd": (_i32, [_vp, _vp, _i64, _vp, _i64, _vp, _i64, _i32, _i32, ctypes.POINTER(GemmEpi), _vp, _vp]),
    "sr_attention_key_box": (_i32, [_vp, _vp, _i64, _i32, _i64, _i32, _i32, _vp, _vp, _vp]),
    "sr_attention_key_box_scratch": (_i32, [_i32, _i32, _i32]),
    "sr_qk_bwd_workspace_floats": (_i64, [_i32, _i32]),
    "sr_qk_bwd_f32": (_i32, [_vp, _vp, _i64, _vp, _i64, _vp, _i64, _i32, _i32, ctypes.POINTER(GemmEpi), _vp, _vp]),
    "sr_cast_bf16": (_i32, [_vp, _vp, _i64, _vp, _i64, _i32, _i32, _f32]),
    "sr_weight_refresh_bf16": (_i32, [_vp, _i32, _vp]),
    "sr_weight_refresh_plan": (_i32, [_i32, _vp, _vp]),
    "sr_weight_refresh_list_bf16": (_i32, [_vp, _i32, _vp, _vp, _i32]),
    "sr_nonfinite_check": (_i32, [_vp, _vp, _i64, _vp, _vp]),
    "sr_adam_f32": (_i32, [_vp, _vp, _vp, _vp, _vp, _i64, _f32, _f32, _f32, _f32, _f32, _i32, _vp, _vp]),
    "sr_transpose_f32": (_i32, [_vp, _i32, _vp, _i64, _i32, _i32, _vp, _vp, _i64]),
    "sr_wgrad_small_f32": (_i32, [_vp, _vp, _i64, _vp, _i64, _vp, _i64, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _i64,
                                  _vp, _vp]),
    "sr_attention_bwd_small_f32": (_i32, [_vp, _vp, _vp, _vp, _i64, _vp, _i64, _vp, _vp, _vp, _i64, _i32, _i32, _i32,
                                          _f32, _i32, _i32, _vp]),
    "sr_adaln_bwd_f32": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _i32, _i32]),
    "sr_act_bwd_f32": (_i32, [_vp, _i32, _vp, _vp, _vp, _i64]),
    "sr_vec_fma_f32": (_i32, [_vp, _vp, _vp, _vp, _i32]),
    "sr_vec_fma2_f32": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _i32]),
    "sr_colsum_fma": (_i32, [_vp, _i32, _vp, _i64, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _i64]),
    "sr_scatter_rows_f32": (_i32, [_vp, _vp, _i64, _vp, _vp, _i64, _i32, _i32, _i32]),
    "sr_copy2d_f32": (_i32, [_vp, _vp, _i64, _vp, _i64, _i32, _i32, _i32]),
    "sr_imc_loss_workspace": (_i64, [_i32, _i32, _i32, _i32, _i32]),
    "sr_imc_loss": (_i32, [_vp, ctypes.POINTER(ImcLossDesc)]),
    "sr_pose_act_bwd_f32": (_i32, [_vp, _vp, _vp, _vp, _i32, _i32]),
    "sr_resize_crop_chw_f32": (_i32, [_vp, _vp, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _vp]),
}
EXPORTED = tuple(_PROTOS)


# oldest library ABI (sr_version, major << 16 | minor) whose entry points these bindings call correctly
ABI_MIN = 1 << 16


class SfmAmdError(RuntimeError):
    pass


_lib = None


def load(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load (once) and return the library; raise if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise SfmAmdError(
            f"libsfm_amd.so not found at {path}: build it with `make -C self-supervise-sfm_amd/csrc` "
            "(there is no CPU fallback)")
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    # an SFM_AMD_LIB override (an older build for a same-box A/B) may lack newer entry points: they
    # stay unbound and fail if called; the in-tree library must export every one.  A build older
    # than ABI_MIN is refused: its existing entry points take structs / arguments that changed
    # meaning in 1.0 (GemmEpi.q_scale / q_cols, AttnDesc.q_scaled, sr_colsum's workspace), which an
    # older library would silently ignore
    override = bool(os.environ.get("SFM_AMD_LIB"))
    lib.sr_version.restype = ctypes.c_int32
    lib.sr_version.argtypes = []
    ver = lib.sr_version()
    if ver < ABI_MIN:
        raise SfmAmdError(f"{path}: ABI {ver >> 16}.{ver & 0xFFFF} is older than the {ABI_MIN >> 16}."
                          f"{ABI_MIN & 0xFFFF} these bindings need")
    for name, (res, args) in _PROTOS.items():
        try:
            fn = getattr(lib, name)
        except AttributeError:
            if override:
                continue
            raise
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().sr_last_error().decode(errors="replace")
        raise SfmAmdError(f"{what} failed ({rc}): {msg}")
