"""Deterministic synthetic weights for the SailRecon hot path.

Pretrained weights (``sailrecon.pt``, fetched from a URL by
``train/demo_imc_forward.py:28-32``) are not available offline, so parity
fixtures, tests and the benchmark all use weights produced by ONE seeded rule:

    for every state_dict key (any order):
        g = torch.Generator().manual_seed(zlib.crc32(key))
        value = torch.randn(shape, generator=g) * scale(kind) + offset(kind)

The rule depends only on the key name and shape, so the reference model
(golden-vector generation, ``tests/golden/make_golden.py``) and this
framework's model (which mirrors the reference ``state_dict`` names, SURVEY
§8(b)) receive bit-identical parameters.

Scales are chosen so every stack changes the residual stream visibly (larger
LayerScale gammas than the 0.01 init) and so the FoV ReLU
(``camera_head.py:36``, ``head_act.py:57-58``) stays positive, which keeps the
decoded intrinsics finite (SURVEY §7 "Random-weight degeneracy").
"""

from __future__ import annotations

import math
import zlib
from typing import Dict, Iterable, Tuple

import torch


def _gen(key: str) -> torch.Generator:
    return torch.Generator().manual_seed(zlib.crc32(key.encode("utf-8")))


def synth_param(key: str, shape: Tuple[int, ...]) -> torch.Tensor:
    """Return the synthetic fp32 tensor for one state_dict entry."""
    shape = tuple(int(s) for s in shape)
    g = _gen(key)
    r = torch.randn(shape, generator=g, dtype=torch.float32)
    leaf = key.rsplit(".", 1)[-1]

    if leaf == "gamma":  # LayerScale (layer_scale.py:20)
        return 0.2 + 0.05 * r
    parent = key.rsplit(".", 2)[-2] if "." in key else ""
    if "norm" in parent:
        # LayerNorm affine params: norm1/norm2/q_norm/k_norm/norm/token_norm/trunk_norm
        if leaf == "weight":
            return 1.0 + 0.1 * r
        if leaf == "bias":
            return 0.05 * r
    if key == "camera_head.pose_branch.fc2.bias" or key.endswith("pose_branch.fc2.bias"):
        # keep translation small, quaternion near identity (xyzw), FoV positive
        v = 0.02 * r
        v[3:7] += torch.tensor([0.0, 0.0, 0.0, 1.0])[: max(0, min(4, shape[0] - 3))]
        if shape[0] >= 9:
            v[7:9] += 1.0
        return v
    if key.endswith("pose_branch.fc2.weight"):
        return 0.002 * r
    if leaf == "bias":
        return 0.02 * r
    if leaf == "weight" and len(shape) >= 2:
        fan_in = int(math.prod(shape[1:]))
        return r / math.sqrt(fan_in)
    if leaf in ("camera_token", "register_token", "camera_token_reloc",
                "register_token_reloc", "cls_token", "register_tokens", "mask_token"):
        return 0.5 * r
    if leaf == "pos_embed":
        return 0.1 * r
    if leaf == "empty_pose_tokens":
        return 0.5 * r
    return 0.02 * r


def synth_state_dict(named_shapes: Iterable[Tuple[str, Tuple[int, ...]]]) -> Dict[str, torch.Tensor]:
    """Build a full state_dict from ``(key, shape)`` pairs."""
    return {k: synth_param(k, s) for k, s in named_shapes}


def synth_state_dict_like(module: torch.nn.Module) -> Dict[str, torch.Tensor]:
    """Synthetic state_dict with the keys/shapes of ``module.state_dict()``."""
    return synth_state_dict((k, tuple(v.shape)) for k, v in module.state_dict().items())
