"""Pose encoding <-> camera matrices (reference: sailrecon/utils/pose_enc.py:68-135).

On a ROCm device the decode runs in the sr_pose_decode_f32 kernel; CPU tensors use
the same formulas in torch (API compatibility for callers outside the hot path).
"""

import torch

from .rotation import quat_to_mat


def pose_encoding_to_extri_intri(pose_encoding, image_size_hw=None, pose_encoding_type="absT_quaR_FoV",
                                 build_intrinsics=True):
    if pose_encoding_type != "absT_quaR_FoV":
        raise NotImplementedError
    if pose_encoding.is_cuda and build_intrinsics and pose_encoding.dtype == torch.float32:
        from .. import ops
        lead = pose_encoding.shape[:-1]
        enc = pose_encoding.reshape(-1, 9).contiguous()
        ext = torch.empty(enc.shape[0], 3, 4, device=enc.device, dtype=torch.float32)
        intr = torch.empty(enc.shape[0], 3, 3, device=enc.device, dtype=torch.float32)
        ops.pose_decode(enc, image_size_hw, ext, intr)
        return ext.view(*lead, 3, 4), intr.view(*lead, 3, 3)
    T, quat = pose_encoding[..., :3], pose_encoding[..., 3:7]
    fov_h, fov_w = pose_encoding[..., 7], pose_encoding[..., 8]
    extrinsics = torch.cat([quat_to_mat(quat), T[..., None]], dim=-1)
    intrinsics = None
    if build_intrinsics:
        H, W = image_size_hw
        fy = (H / 2.0) / torch.tan(fov_h / 2.0)
        fx = (W / 2.0) / torch.tan(fov_w / 2.0)
        intrinsics = torch.zeros(pose_encoding.shape[:2] + (3, 3), device=pose_encoding.device)
        intrinsics[..., 0, 0] = fx
        intrinsics[..., 1, 1] = fy
        intrinsics[..., 0, 2] = W / 2
        intrinsics[..., 1, 2] = H / 2
        intrinsics[..., 2, 2] = 1.0
    return extrinsics, intrinsics
