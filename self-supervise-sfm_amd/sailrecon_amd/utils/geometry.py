"""Depth unprojection — drop-in for sailrecon/utils/geometry.py:19-130.

``unproject_depth_points`` runs on device (sr_unproject_depth_f32).
``unproject_depth_map_to_point_map`` keeps the reference's contract: it returns a numpy array
of world points [S, H, W, 3] in float64, which the reference produces from its float64
closed-form SE(3) inverse (geometry.py:132-186).  The arithmetic here is fp32 on the GPU;
only the result is copied to the host.
"""

from __future__ import annotations

import numpy as np
import torch

from .. import ops, runtime


def unproject_depth_points(depth_map: torch.Tensor, extrinsics_cam: torch.Tensor,
                           intrinsics_cam: torch.Tensor) -> torch.Tensor:
    """depth [S, H, W] or [S, H, W, 1], extrinsic [S, 3, 4] (cam from world, OpenCV),
    intrinsic [S, 3, 3] (zero skew) -> world points [S, H, W, 3] fp32 on device."""
    runtime.require_device(depth_map, "unproject_depth_points")
    d = depth_map.detach().float()
    if d.dim() == 4:
        d = d.squeeze(-1)
    d = d.contiguous()
    S, H, W = d.shape
    e = extrinsics_cam.detach().float().reshape(S, 3, 4).contiguous()
    k = intrinsics_cam.detach().float().reshape(S, 3, 3).contiguous()
    out = torch.empty(S, H, W, 3, device=d.device, dtype=torch.float32)
    ops.unproject_depth(d, e, k, out)
    return out


def unproject_depth_map_to_point_map(depth_map, extrinsics_cam, intrinsics_cam) -> np.ndarray:
    """Reference-compatible wrapper: same arguments, numpy float64 [S, H, W, 3] result."""
    pts = unproject_depth_points(depth_map, extrinsics_cam, intrinsics_cam)
    return pts.cpu().numpy().astype(np.float64)
