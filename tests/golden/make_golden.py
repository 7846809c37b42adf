"""Generate golden vectors by running the REAL reference (read-only import).

Run in the build container only (``/root/reference`` does not exist on the GPU
box):   PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

Weights: the seeded rule in ``sailrecon_amd/utils/synth_weights.py`` applied to
the reference modules' own state_dict keys.  Inputs: seeded ``torch.rand``.
Subsample draws: the reference's own ``Aggregator.generator`` re-seeded with
``manual_seed(0)``; the indices it drew are replayed and stored too.

Outputs (numpy .npz, no pickle):
  g1_small_56.npz, g1_small_70.npz  small-config end-to-end (full tensors)
  g2_blocks.npz                     block KATs at real width (C=1024 / 2048)
  g3_ops.npz                        op KATs (RoPE, masks)
  g4_c1_224.npz                     full-size config 1 (N=2 @ 224) summaries
  g5_518_n1.npz                     full-size N=1 @ 518 summaries
  g9_518_n8.npz, g10_518_n32.npz    full-size BASELINE C2 / C3 summaries (args c2, c3)
  g11_small_interleaved.npz         small config, permuted + interleaved anchor/query lists
  state_dict_keys.json              reference state_dict keys + shapes
"""

from __future__ import annotations

import json
import os
import sys
import time
from functools import partial

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "self-supervise-sfm_amd"))
sys.path.insert(0, "/root/reference")
sys.dont_write_bytecode = True

from sailrecon_amd.utils.synth_weights import synth_state_dict_like  # noqa: E402

from sailrecon.heads.camera_head import CameraHead, build_lr_mask  # noqa: E402
from sailrecon.layers.attention import MemEffAttention  # noqa: E402
from sailrecon.layers.block import Block  # noqa: E402
from sailrecon.layers.rope import RotaryPositionEmbedding2D  # noqa: E402
from sailrecon.models.aggregator import Aggregator, build_allow_block, expand_to_token  # noqa: E402
from sailrecon.utils.pose_enc import pose_encoding_to_extri_intri  # noqa: E402

torch.set_num_threads(8)


def np32(t):
    return t.detach().float().cpu().numpy().astype(np.float32)


def replay_indices(seed, depth, na, n_patch, rank):
    g = torch.Generator().manual_seed(seed)
    out = np.zeros((depth, na, rank), dtype=np.int64)
    for l in range(depth):
        for a in range(na):
            out[l, a] = torch.randperm(n_patch, generator=g)[:rank].numpy()
    return out


class Hot(torch.nn.Module):
    """aggregator + camera_head with the reference module names (sail_recon.py:38-45)."""

    def __init__(self, agg_kw, cam_kw):
        super().__init__()
        self.aggregator = Aggregator(**agg_kw)
        self.camera_head = CameraHead(**cam_kw)


def run_hot(model, images, na, fix_rank, seed=0, lists=None):
    S = images.shape[1]
    no_reloc, reloc = lists if lists is not None else (list(range(na)), list(range(na, S)))
    model.aggregator.generator.manual_seed(seed)
    with torch.no_grad():
        feats, psi, cam_last = model.aggregator(images, no_reloc, reloc, fix_rank=fix_rank)  # sail_recon.py:101
        poses = model.camera_head(feats, cam_last)  # sail_recon.py:121
        ext, intr = pose_encoding_to_extri_intri(poses[-1], (images.shape[-2], images.shape[-1]))
    return feats, psi, cam_last, poses, ext, intr


def small_case(tag, img, n_views, fix_rank):
    torch.manual_seed(0)
    agg_kw = dict(img_size=56, patch_size=14, embed_dim=384, depth=2, num_heads=6,
                  patch_embed="dinov2_vits14_reg", intermediate_layer_idx=[0, 1])
    cam_kw = dict(dim_in=768, trunk_depth=2, num_heads=6)
    m = Hot(agg_kw, cam_kw).eval()
    m.load_state_dict(synth_state_dict_like(m))
    g = torch.Generator().manual_seed(1)
    x = torch.rand(1, n_views, 3, img, img, generator=g)
    images = torch.cat([x, x], dim=1)
    feats, psi, cam_last, poses, ext, intr = run_hot(m, images, n_views, fix_rank)
    n_patch = (img // 14) ** 2
    rank = min(fix_rank, n_patch)
    d = dict(images=np32(images), fix_rank=np.int64(fix_rank), n_views=np.int64(n_views),
             sub_idx=replay_indices(0, 2, n_views, n_patch, rank),
             feat_0=np32(feats[0]), feat_1=np32(feats[1]), cam_token_last_layer=np32(cam_last),
             pose_enc=np.stack([np32(p) for p in poses]), extrinsic=np32(ext), intrinsic=np32(intr))
    np.savez_compressed(os.path.join(HERE, f"g1_small_{tag}.npz"), **d)
    print("wrote", tag, {k: v.shape for k, v in d.items()})
    with open(os.path.join(HERE, "small_state_dict_keys.json"), "w") as f:
        json.dump({k: list(v.shape) for k, v in m.state_dict().items()}, f, indent=0, sort_keys=True)
    return m


def interleaved_case():
    """Frame-order semantics (aggregator.py:287-299,351-399): anchors and queries interleaved and
    permuted, frame 0 a query (so no anchor gets camera_token[:, 0])."""
    torch.manual_seed(0)
    agg_kw = dict(img_size=56, patch_size=14, embed_dim=384, depth=2, num_heads=6,
                  patch_embed="dinov2_vits14_reg", intermediate_layer_idx=[0, 1])
    cam_kw = dict(dim_in=768, trunk_depth=2, num_heads=6)
    m = Hot(agg_kw, cam_kw).eval()
    m.load_state_dict(synth_state_dict_like(m))
    g = torch.Generator().manual_seed(5)
    images = torch.rand(1, 6, 3, 56, 56, generator=g)
    no_reloc, reloc = [3, 1, 4], [0, 5, 2]
    feats, psi, cam_last, poses, ext, intr = run_hot(m, images, 3, 10, lists=(no_reloc, reloc))
    d = dict(images=np32(images), fix_rank=np.int64(10), no_reloc=np.array(no_reloc), reloc=np.array(reloc),
             sub_idx=replay_indices(0, 2, 3, 16, 10),
             feat_0=np32(feats[0]), feat_1=np32(feats[1]), cam_token_last_layer=np32(cam_last),
             pose_enc=np.stack([np32(p) for p in poses]), extrinsic=np32(ext), intrinsic=np32(intr))
    np.savez_compressed(os.path.join(HERE, "g11_small_interleaved.npz"), **d)
    print("wrote g11_small_interleaved", {k: v.shape for k, v in d.items()})


def block_kats():
    out = {}
    g = torch.Generator().manual_seed(2)
    # aggregator-style block (aggregator.py:99-114)
    rope = RotaryPositionEmbedding2D(frequency=100)
    blk = Block(dim=1024, num_heads=16, init_values=0.01, qk_norm=True, rope=rope).eval()
    blk.load_state_dict(synth_state_dict_like(blk))
    x = torch.randn(2, 37, 1024, generator=g)
    pos = torch.randint(0, 38, (2, 37, 2), generator=g)
    pos[:, :5] = 0
    with torch.no_grad():
        out["agg_x"], out["agg_pos"], out["agg_y"] = np32(x), pos.numpy(), np32(blk(x, pos=pos))
    keys = {"agg": {k: list(v.shape) for k, v in blk.state_dict().items()}}
    # DINO-style block (vision_transformer.py:105,161-177; MemEffAttention)
    blk = Block(dim=1024, num_heads=16, init_values=1.0, norm_layer=partial(torch.nn.LayerNorm, eps=1e-6),
                attn_class=MemEffAttention).eval()
    blk.load_state_dict(synth_state_dict_like(blk))
    x = torch.randn(2, 37, 1024, generator=g)
    with torch.no_grad():
        out["dino_x"], out["dino_y"] = np32(x), np32(blk(x))
    keys["dino"] = {k: list(v.shape) for k, v in blk.state_dict().items()}
    # camera trunk block (camera_head.py:51-61) with ~build_lr_mask (camera_head.py:165)
    blk = Block(dim=2048, num_heads=16, init_values=0.01).eval()
    blk.load_state_dict(synth_state_dict_like(blk))
    x = torch.randn(1, 10, 2048, generator=g)
    mask = ~build_lr_mask(10, [0, 1, 2, 3, 4])
    with torch.no_grad():
        out["cam_x"], out["cam_mask"], out["cam_y"] = np32(x), mask.numpy(), np32(blk(x, None, mask))
    keys["cam"] = {k: list(v.shape) for k, v in blk.state_dict().items()}
    np.savez_compressed(os.path.join(HERE, "g2_blocks.npz"), **out)
    with open(os.path.join(HERE, "block_state_dict_keys.json"), "w") as f:
        json.dump(keys, f, indent=0, sort_keys=True)
    print("wrote g2_blocks")


def op_kats():
    g = torch.Generator().manual_seed(3)
    rope = RotaryPositionEmbedding2D(frequency=100)
    t = torch.randn(1, 16, 261, 64, generator=g)
    pos = torch.randint(0, 17, (1, 261, 2), generator=g)
    allow = build_allow_block(4, [0, 1], [2, 3])
    full = expand_to_token(allow, 3)
    d = dict(rope_in=np32(t), rope_pos=pos.numpy(), rope_out=np32(rope(t, pos)),
             allow_4_2=allow.numpy(), allow_tok=full.numpy(),
             lr_mask_6_3=build_lr_mask(6, [0, 1, 2]).numpy())
    np.savez_compressed(os.path.join(HERE, "g3_ops.npz"), **d)
    print("wrote g3_ops")


def summarize(feats, cam_last, poses, ext, intr, rows):
    d = dict(cam_token_last_layer=np32(cam_last), pose_enc=np.stack([np32(p) for p in poses]),
             extrinsic=np32(ext), intrinsic=np32(intr), sample_rows=rows)
    for k, v in feats.items():
        if k < 0:
            continue
        v = v[0]  # [Nq, P, 2C]
        d[f"feat_{k}_rownorm"] = np32(v.norm(dim=-1))
        d[f"feat_{k}_cam"] = np32(v[:, 0])
        d[f"feat_{k}_rows"] = np32(v.reshape(-1, v.shape[-1])[torch.as_tensor(rows)])
    return d


def full_case(fname, img, n_views, fix_rank=300):
    t0 = time.time()
    torch.manual_seed(0)
    m = Hot(dict(img_size=518, patch_size=14, embed_dim=1024), dict(dim_in=2048)).eval()
    sd = synth_state_dict_like(m)
    m.load_state_dict(sd)
    del sd
    keys = {k: list(v.shape) for k, v in m.state_dict().items()}
    g = torch.Generator().manual_seed(n_views)
    x = torch.rand(n_views, 3, img, img, generator=g)
    images = torch.cat([x, x])[None]  # demo_imc_forward.py:76-82
    t1 = time.time()
    feats, psi, cam_last, poses, ext, intr = run_hot(m, images, n_views, fix_rank)
    t2 = time.time()
    n_patch = (img // 14) ** 2
    P = n_patch + 5
    rows = np.random.default_rng(0).choice(n_views * P, size=min(48, n_views * P), replace=False)
    rows = np.sort(np.concatenate([rows, [0, P - 1]])).astype(np.int64)
    d = summarize(feats, cam_last, poses, ext, intr, rows)
    d.update(n_views=np.int64(n_views), img=np.int64(img), fix_rank=np.int64(fix_rank),
             sub_idx=replay_indices(0, 24, n_views, n_patch, min(fix_rank, n_patch)),
             ref_forward_s=np.float64(t2 - t1))
    np.savez_compressed(os.path.join(HERE, fname), **d)
    print(f"wrote {fname}: build {t1 - t0:.1f}s forward {t2 - t1:.1f}s")
    return keys


if __name__ == "__main__":
    which = sys.argv[1:] or ["small", "blocks", "ops", "c1", "518"]
    if "small" in which:
        small_case("56", 56, 2, 10)
        small_case("70", 70, 3, 10)
    if "small5" in which:  # 5 anchors + 5 queries: uneven frame sharding over 2 / 3 ranks
        small_case("56_n5", 56, 5, 10)
    if "small9" in which:  # 9 anchors + 9 queries: frame sharding over 8 ranks (2,1,1,1,1,1,1,1)
        small_case("56_n9", 56, 9, 10)
    if "blocks" in which:
        block_kats()
    if "ops" in which:
        op_kats()
    if "c1" in which:
        keys = full_case("g4_c1_224.npz", 224, 2)
        with open(os.path.join(HERE, "state_dict_keys.json"), "w") as f:
            json.dump(keys, f, indent=0, sort_keys=True)
    if "518" in which:
        full_case("g5_518_n1.npz", 518, 1)
    if "c2" in which:  # BASELINE config 2: N=8 @518 (~2 min on 8 cores)
        full_case("g9_518_n8.npz", 518, 8)
    if "c3" in which:  # BASELINE config 3: N=32 @518 (~17 min, ~30 GB RSS on 8 cores)
        full_case("g10_518_n32.npz", 518, 32)
    if "interleaved" in which:
        interleaved_case()
