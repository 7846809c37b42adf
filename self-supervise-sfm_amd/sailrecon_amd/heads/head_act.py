"""Pose / head activations (reference: sailrecon/heads/head_act.py:12-127).

Host-side torch mirrors for API compatibility; on the hot path activate_pose is
fused into the sr_pose_update_f32 kernel (camera_head.py:178-184).
"""

import torch
import torch.nn.functional as F


def activate_pose(pred_pose_enc, trans_act="linear", quat_act="linear", fl_act="linear"):
    T, quat, fl = pred_pose_enc[..., :3], pred_pose_enc[..., 3:7], pred_pose_enc[..., 7:]
    return torch.cat([base_pose_act(T, trans_act), base_pose_act(quat, quat_act), base_pose_act(fl, fl_act)], dim=-1)


def base_pose_act(pose_enc, act_type="linear"):
    if act_type == "linear":
        return pose_enc
    if act_type == "inv_log":
        return inverse_log_transform(pose_enc)
    if act_type == "exp":
        return torch.exp(pose_enc)
    if act_type == "relu":
        return F.relu(pose_enc)
    raise ValueError(f"Unknown act_type: {act_type}")


def inverse_log_transform(y):
    return torch.sign(y) * torch.expm1(torch.abs(y))
