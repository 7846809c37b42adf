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


# DPT head fixtures (tests/golden/make_golden_dpt.py)
DPT_SMALL = dict(dim_in=256, patch_size=14, features=64, out_channels=[32, 64, 128, 128],
                 intermediate_layer_idx=[0, 1, 2, 3])
DPT_HEADS = {"point": dict(output_dim=4, activation="inv_log", conf_activation="expp1"),
             "depth": dict(output_dim=2, activation="exp", conf_activation="expp1")}


def dpt_tokens(layers, S, P, C, seed):
    """The generator's seeded token maps (make_golden_dpt.tokens_for)."""
    g = torch.Generator().manual_seed(seed)
    return {l: torch.randn(1, S, P, C, generator=g) for l in layers}


def dpt_224_inputs():
    toks = dpt_tokens([4, 11, 17, 23], 2, 5 + 16 * 16, 2048, 3)
    images = torch.rand(1, 2, 3, 224, 224, generator=torch.Generator().manual_seed(4))
    return toks, images


def dpt_small_model_sd(kind):
    """(reference-named) rule state_dict of the small DPT config, keys from our mirror module."""
    from sailrecon_amd.heads.dpt_head import DPTHead
    from sailrecon_amd.utils.synth_weights import synth_state_dict_like
    m = DPTHead(**DPT_SMALL, **DPT_HEADS[kind])
    return m, synth_state_dict_like(m)
