"""Helpers shared by the parity tests: load fixtures, rebuild rule weights."""

import json
import os

import numpy as np
import torch

from sailrecon_amd.utils.synth_weights import synth_state_dict

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_npz(name):
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def key_shapes(name, section=None):
    with open(os.path.join(GOLDEN, name)) as f:
        d = json.load(f)
    if section is not None:
        d = d[section]
    return [(k, tuple(v)) for k, v in sorted(d.items())]


def rule_state_dict(name, section=None, prefix=""):
    return {prefix + k: v for k, v in synth_state_dict(key_shapes(name, section)).items()}


def rel_l2(a, b):
    a = torch.as_tensor(np.asarray(a), dtype=torch.float64)
    b = torch.as_tensor(np.asarray(b), dtype=torch.float64)
    return float((a - b).norm() / b.norm().clamp_min(1e-12))


SMALL_AGG = dict(patch=14, embed_dim=384, depth=2, heads=6, dino_depth=12, dino_heads=6, inter_idx=(0, 1))
SMALL_CAM = dict(cam_heads=6, cam_depth=2)
