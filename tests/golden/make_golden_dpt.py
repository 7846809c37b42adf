"""Golden vectors for the DPT point / depth heads and the depth unprojection (SURVEY §8(f)
rank 1), produced by running the REAL reference modules (read-only import).

Build container only (``/root/reference`` is absent on the GPU box):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_dpt.py

Weights: the seeded rule (``sailrecon_amd/utils/synth_weights.py``) on the reference
DPTHead's own state_dict keys.  Inputs: seeded randn tokens / rand images.

  g6_dpt_small.npz   DPTHead(dim_in=256, features=64, out_channels=[32,64,128,128]) on a
                     56x70 image (4x5 patches), S=3 frames, frames_chunk_size=2;
                     point (inv_log / expp1, 4 channels) and depth (exp / expp1, 2 channels)
  g6_dpt_224.npz     default DPTHead(dim_in=2048) point + depth heads at 224x224, S=2
  g6_unproject.npz   unproject_depth_map_to_point_map on the 224 depth maps with random
                     cameras (geometry.py:19-130)
  dpt_state_dict_keys.json
  g6_dpt_feat_small.npz  DPTHead(SMALL, feature_only=True) (dpt_head.py:123-126,286-287):
                     the fused feature map [1, S, 64, H, W], frames_chunk_size=2
                     (``--only feature`` writes this file alone)
"""

from __future__ import annotations

import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "self-supervise-sfm_amd"))
sys.path.insert(0, "/root/reference")
sys.dont_write_bytecode = True

from sailrecon_amd.utils.synth_weights import synth_state_dict_like  # noqa: E402

from sailrecon.heads.dpt_head import DPTHead  # noqa: E402
from sailrecon.utils.geometry import unproject_depth_map_to_point_map  # noqa: E402

torch.set_num_threads(8)

SMALL = dict(dim_in=256, patch_size=14, features=64, out_channels=[32, 64, 128, 128],
             intermediate_layer_idx=[0, 1, 2, 3])
HEADS = {"point": dict(output_dim=4, activation="inv_log", conf_activation="expp1"),
         "depth": dict(output_dim=2, activation="exp", conf_activation="expp1")}


def build(cfg, kind):
    m = DPTHead(**cfg, **HEADS[kind]).eval()
    m.load_state_dict(synth_state_dict_like(m))
    return m


def tokens_for(layers, S, P, C, seed):
    g = torch.Generator().manual_seed(seed)
    return {l: torch.randn(1, S, P, C, generator=g) for l in layers}


def feature_only():
    S, H, W = 3, 56, 70
    P = 5 + (H // 14) * (W // 14)
    toks = tokens_for(SMALL["intermediate_layer_idx"], S, P, SMALL["dim_in"], 5)
    images = torch.rand(1, S, 3, H, W, generator=torch.Generator().manual_seed(6))
    m = DPTHead(**SMALL, feature_only=True).eval()
    m.load_state_dict(synth_state_dict_like(m))
    with torch.no_grad():
        feat = m(toks, images=images, patch_start_idx=5, frames_chunk_size=2)
    out = dict(images=images.numpy(), feat=feat.numpy())
    for l, t in toks.items():
        out[f"tok_{l}"] = t.numpy()
    np.savez(os.path.join(HERE, "g6_dpt_feat_small.npz"), **out)


def main():
    out = {}
    # ---- small config
    S, H, W = 3, 56, 70
    P = 5 + (H // 14) * (W // 14)
    toks = tokens_for(SMALL["intermediate_layer_idx"], S, P, SMALL["dim_in"], 1)
    images = torch.rand(1, S, 3, H, W, generator=torch.Generator().manual_seed(2))
    small = dict(images=images.numpy())
    for l, t in toks.items():
        small[f"tok_{l}"] = t.numpy()
    with torch.no_grad():
        for kind in HEADS:
            preds, conf = build(SMALL, kind)(toks, images=images, patch_start_idx=5, frames_chunk_size=2)
            small[f"{kind}_preds"] = preds.numpy()
            small[f"{kind}_conf"] = conf.numpy()
    np.savez(os.path.join(HERE, "g6_dpt_small.npz"), **small)

    # ---- full width at 224
    S, H, W = 2, 224, 224
    P = 5 + (H // 14) * (W // 14)
    layers = [4, 11, 17, 23]
    toks = tokens_for(layers, S, P, 2048, 3)
    images = torch.rand(1, S, 3, H, W, generator=torch.Generator().manual_seed(4))
    full = {}  # tokens / images are regenerated from their seeds by the tests (tokens_for(...) above)
    keys = {}
    with torch.no_grad():
        for kind in HEADS:
            m = build(dict(dim_in=2048), kind)
            keys[kind] = {k: list(v.shape) for k, v in m.state_dict().items()}
            preds, conf = m(toks, images=images, patch_start_idx=5)
            full[f"{kind}_preds"] = preds.numpy()
            full[f"{kind}_conf"] = conf.numpy()
    np.savez(os.path.join(HERE, "g6_dpt_224.npz"), **full)
    with open(os.path.join(HERE, "dpt_state_dict_keys.json"), "w") as f:
        json.dump(keys, f, indent=0)

    # ---- unprojection of the 224 depth maps with random cameras
    g = torch.Generator().manual_seed(5)
    q = torch.randn(S, 4, generator=g)
    q = q / q.norm(dim=-1, keepdim=True)
    x, y, z, w_ = q.unbind(-1)
    R = torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - z * w_), 2 * (x * z + y * w_),
                     2 * (x * y + z * w_), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w_),
                     2 * (x * z - y * w_), 2 * (y * z + x * w_), 1 - 2 * (x * x + y * y)], -1).view(S, 3, 3)
    t = torch.randn(S, 3, 1, generator=g)
    extr = torch.cat([R, t], -1)
    f = 150.0 + 20.0 * torch.rand(S, generator=g)
    intr = torch.zeros(S, 3, 3)
    intr[:, 0, 0], intr[:, 1, 1] = f, f * 1.05
    intr[:, 0, 2], intr[:, 1, 2], intr[:, 2, 2] = W / 2, H / 2, 1.0
    depth = torch.from_numpy(full["depth_preds"][0])  # [S, H, W, 1]
    pts = unproject_depth_map_to_point_map(depth, extr, intr)
    np.savez(os.path.join(HERE, "g6_unproject.npz"), depth=depth.numpy(), extrinsic=extr.numpy(),
             intrinsic=intr.numpy(), points=np.asarray(pts, dtype=np.float32))
    for name in ("g6_dpt_small.npz", "g6_dpt_224.npz", "g6_unproject.npz"):
        print(name, os.path.getsize(os.path.join(HERE, name)) // 1024, "KiB")


if __name__ == "__main__":
    if sys.argv[1:] == ["--only", "feature"]:
        feature_only()
    else:
        main()
        feature_only()
