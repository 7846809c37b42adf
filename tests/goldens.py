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


def dpt_feat_model_sd():
    """The small DPT config with feature_only=True (dpt_head.py:123-126) and its rule state_dict."""
    from sailrecon_amd.heads.dpt_head import DPTHead
    from sailrecon_amd.utils.synth_weights import synth_state_dict_like
    m = DPTHead(**DPT_SMALL, feature_only=True)
    return m, synth_state_dict_like(m)


# ---------------------------------------------------------------- input formation (§8(f) rank 2)
def pil_process_reference(arr, target, is_depth):
    """train/utils/io.py:118-153 step by step with Pillow, which is what the reference calls
    (torchvision's ToTensor is uint8 -> float / 255).  Returns [1, C, T, T] fp32 (host)."""
    from PIL import Image
    img = Image.fromarray(arr) if is_depth else Image.fromarray(arr).convert("RGB")
    w, h = img.size
    m = max(w, h)
    if m != w or m != h:
        sq = Image.new(img.mode, (m, m), color=0)
        sq.paste(img, ((m - w) // 2, (m - h) // 2))
        img = sq
    img = img.resize((target, target), Image.Resampling.BICUBIC)
    a = np.array(img)
    if is_depth:
        return torch.from_numpy(a.astype(np.float32) / 1000)[None][None]
    return torch.from_numpy(a).permute(2, 0, 1).float().div(255)[None]


def pil_load_reference(images, mode=None, square_target=None):
    """sailrecon/utils/load_fn.py:13-96 (square_target set) or :99-240 (mode "crop"/"pad") with
    Pillow + torch on the host, on PIL images instead of paths."""
    from PIL import Image
    T = 518
    outs, coords = [], []
    for img in images:
        if img.mode == "RGBA":
            bg = Image.new("RGBA", img.size, (255, 255, 255, 255))
            img = Image.alpha_composite(bg, img)
        img = img.convert("RGB")
        w, h = img.size
        if square_target is not None:
            m = max(w, h)
            left, top = (m - w) // 2, (m - h) // 2
            s = square_target / m
            coords.append(np.array([left * s, top * s, (left + w) * s, (top + h) * s, w, h]))
            sq = Image.new("RGB", (m, m), (0, 0, 0))
            sq.paste(img, (left, top))
            sq = sq.resize((square_target, square_target), Image.Resampling.BICUBIC)
            outs.append(torch.from_numpy(np.array(sq)).permute(2, 0, 1).float().div(255))
            continue
        if mode == "pad" and w < h:
            nh, nw = T, round(w * (T / h) / 14) * 14
        else:
            nw, nh = T, round(h * (T / w) / 14) * 14
        t = torch.from_numpy(np.array(img.resize((nw, nh), Image.Resampling.BICUBIC))).permute(2, 0, 1)
        t = t.float().div(255)
        if mode == "crop" and nh > T:
            y0 = (nh - T) // 2
            t = t[:, y0:y0 + T, :]
        if mode == "pad":
            hp, wp = T - t.shape[1], T - t.shape[2]
            if hp > 0 or wp > 0:
                t = torch.nn.functional.pad(t, (wp // 2, wp - wp // 2, hp // 2, hp - hp // 2), value=1.0)
        outs.append(t)
    if square_target is not None:
        return torch.stack(outs), torch.from_numpy(np.array(coords)).float()
    H = max(t.shape[1] for t in outs)
    W = max(t.shape[2] for t in outs)
    padded = []
    for t in outs:
        hp, wp = H - t.shape[1], W - t.shape[2]
        if hp > 0 or wp > 0:
            t = torch.nn.functional.pad(t, (wp // 2, wp - wp // 2, hp // 2, hp - hp // 2), value=1.0)
        padded.append(t)
    return torch.stack(padded)


# Full-model parity bounds, rel-L2 against the reference's fp32 goldens, per quantity class: about
# 2-4x the largest error measured on MI355X over every golden, sharded run and residual mode (each
# test prints what it measured: "PARITY ..." lines in the GPU logs, profiles/r05_*gputests*.log),
# never above SURVEY §8(c)'s 2e-2 (bf16) or the north star's 1e-4 (pose, fp32).  Measured round 5
# (c*q rounded once, round-4 kernels otherwise):
#   fp32  feat 2.7e-6 (C3 camera tokens)   pose 3.2e-7 (C3 sharded extrinsic)
#   bf16  feat 4.7e-3 (C3 deferred-residual camera columns of layer 23)   pose 8.1e-4 (N=1 @518 extrinsic)
PARITY_TOL = {"fp32": {"feat": 1e-5, "pose": 1e-5},
              "bf16": {"feat": 1e-2, "pose": 2e-3}}


def parity_tol(key: str, mode: str) -> float:
    """Bound for one checked quantity: pose encodings / extrinsics / intrinsics are the "pose"
    class, feature maps and camera tokens the "feat" class."""
    cls = "pose" if any(t in key for t in ("pose", "extrinsic", "intrinsic")) else "feat"
    return PARITY_TOL[mode][cls]
