"""CPU ORACLE for the SailRecon aggregator + camera-pose head hot path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module, and only as the
checker / the timed CPU baseline.  The product path (``sailrecon_amd``) never
imports it and fails loudly when its HIP library is missing.

What it is: a plain PyTorch-CPU fp32 restatement of the reference algorithm,
written from the reference's behaviour (not copied), functional style over an
explicit ``state_dict``.  It keeps the reference's own op choices, including the
dense boolean reloc mask (``aggregator.py:302-311``) and the scatter
reassembly (``aggregator.py:393-399``), so that it times like the reference CPU
path.

Pinning: checked against golden vectors produced by importing the real
reference in the build container (``tests/golden/make_golden.py``); see
``tests/test_oracle_golden.py``.
"""

from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn.functional as F

Tensor = torch.Tensor
SD = Dict[str, Tensor]

RESNET_MEAN = (0.485, 0.456, 0.406)  # aggregator.py:31
RESNET_STD = (0.229, 0.224, 0.225)  # aggregator.py:32


# --------------------------------------------------------------------------
# layers (sailrecon/layers)
# --------------------------------------------------------------------------

def layer_norm(x: Tensor, w: Optional[Tensor], b: Optional[Tensor], eps: float) -> Tensor:
    return F.layer_norm(x, (x.shape[-1],), w, b, eps)


def rope_tables(half_dim: int, max_pos: int, base: float = 100.0) -> Tuple[Tensor, Tensor]:
    """cos/sin tables, rope.py:93-124 (fp32; angles duplicated cat(a, a))."""
    exps = torch.arange(0, half_dim, 2).float() / half_dim
    inv_freq = 1.0 / (base ** exps)
    pos = torch.arange(max_pos, dtype=inv_freq.dtype)
    ang = torch.einsum("i,j->ij", pos, inv_freq)
    ang = torch.cat((ang, ang), dim=-1)
    return ang.cos(), ang.sin()


def rope2d(t: Tensor, pos: Tensor, base: float = 100.0) -> Tensor:
    """2-D RoPE, rope.py:165-207.  t [B,H,L,D], pos [B,L,2] int (y, x)."""
    half = t.shape[-1] // 2
    cos_t, sin_t = rope_tables(half, int(pos.max()) + 1, base)

    def one(x: Tensor, p: Tensor) -> Tensor:  # rope.py:140-163
        c = F.embedding(p, cos_t)[:, None]
        s = F.embedding(p, sin_t)[:, None]
        x1, x2 = x[..., : half // 2], x[..., half // 2:]
        return x * c + torch.cat((-x2, x1), dim=-1) * s

    ty, tx = t.chunk(2, dim=-1)
    return torch.cat((one(ty, pos[..., 0]), one(tx, pos[..., 1])), dim=-1)


def attention(sd: SD, pre: str, x: Tensor, heads: int, pos: Optional[Tensor] = None,
              mask: Optional[Tensor] = None, qk_norm: bool = False,
              rope_base: Optional[float] = None) -> Tensor:
    """Attention.forward, attention.py:70-122 (fused SDPA branch)."""
    B, N, C = x.shape
    D = C // heads
    qkv = F.linear(x, sd[pre + "qkv.weight"], sd.get(pre + "qkv.bias"))
    q, k, v = qkv.reshape(B, N, 3, heads, D).permute(2, 0, 3, 1, 4).unbind(0)
    if qk_norm:  # attention.py:49-50,78 (LayerNorm(D), eps 1e-5)
        q = layer_norm(q, sd[pre + "q_norm.weight"], sd[pre + "q_norm.bias"], 1e-5)
        k = layer_norm(k, sd[pre + "k_norm.weight"], sd[pre + "k_norm.bias"], 1e-5)
    if rope_base is not None:
        q = rope2d(q, pos, rope_base)
        k = rope2d(k, pos, rope_base)
    o = F.scaled_dot_product_attention(q, k, v, attn_mask=mask)
    o = o.transpose(1, 2).reshape(B, N, C)
    return F.linear(o, sd[pre + "proj.weight"], sd.get(pre + "proj.bias"))


def mlp(sd: SD, pre: str, x: Tensor) -> Tensor:
    """Mlp.forward, mlp.py:34-40 (exact erf GELU)."""
    h = F.gelu(F.linear(x, sd[pre + "fc1.weight"], sd.get(pre + "fc1.bias")))
    return F.linear(h, sd[pre + "fc2.weight"], sd.get(pre + "fc2.bias"))


def block(sd: SD, pre: str, x: Tensor, heads: int, eps: float, pos: Optional[Tensor] = None,
          mask: Optional[Tensor] = None, qk_norm: bool = False,
          rope_base: Optional[float] = None) -> Tensor:
    """Block.forward eval branch, block.py:86-112 (LayerScale layer_scale.py:22-23)."""
    a = attention(sd, pre + "attn.", layer_norm(x, sd[pre + "norm1.weight"], sd[pre + "norm1.bias"], eps),
                  heads, pos, mask, qk_norm, rope_base)
    x = x + a * sd[pre + "ls1.gamma"]
    m = mlp(sd, pre + "mlp.", layer_norm(x, sd[pre + "norm2.weight"], sd[pre + "norm2.bias"], eps))
    return x + m * sd[pre + "ls2.gamma"]


# --------------------------------------------------------------------------
# DINOv2 patch embed (vision_transformer.py, aggregator.py:196-240)
# --------------------------------------------------------------------------

def dino_pos_embed(sd: SD, pre: str, h_img: int, w_img: int, patch: int, npatch: int) -> Tensor:
    """interpolate_pos_encoding, vision_transformer.py:206-240 (antialias, offset 0)."""
    pe = sd[pre + "pos_embed"]
    n0 = pe.shape[1] - 1
    if npatch == n0 and w_img == h_img:
        return pe
    pe = pe.float()
    cls_pe, patch_pe = pe[:, 0], pe[:, 1:]
    dim = pe.shape[-1]
    m = int(math.sqrt(n0))
    # note the reference names the first spatial dim "w" (B, nc, w, h = x.shape)
    out = F.interpolate(patch_pe.reshape(1, m, m, dim).permute(0, 3, 1, 2), mode="bicubic",
                        antialias=True, size=(h_img // patch, w_img // patch))
    out = out.permute(0, 2, 3, 1).view(1, -1, dim)
    return torch.cat((cls_pe.unsqueeze(0), out), dim=1)


def dino_embed(sd: SD, pre: str, img: Tensor, patch: int) -> Tensor:
    """prepare_tokens_with_masks, vision_transformer.py:242-259: patch conv, cls, pos-embed, registers."""
    x = F.conv2d(img, sd[pre + "patch_embed.proj.weight"], sd[pre + "patch_embed.proj.bias"], stride=patch)
    x = x.flatten(2).transpose(1, 2)
    B = x.shape[0]
    x = torch.cat((sd[pre + "cls_token"].expand(B, -1, -1), x), dim=1)
    x = x + dino_pos_embed(sd, pre, img.shape[2], img.shape[3], patch, x.shape[1] - 1)
    reg = sd[pre + "register_tokens"]
    return torch.cat((x[:, :1], reg.expand(B, -1, -1), x[:, 1:]), dim=1)


def dino_forward(sd: SD, pre: str, img: Tensor, patch: int, depth: int, heads: int) -> Tensor:
    """forward_features -> x_norm_patchtokens, vision_transformer.py:242-307."""
    x = dino_embed(sd, pre, img, patch)
    reg = sd[pre + "register_tokens"]
    for i in range(depth):
        x = block(sd, f"{pre}blocks.{i}.", x, heads, 1e-6)
    x = layer_norm(x, sd[pre + "norm.weight"], sd[pre + "norm.bias"], 1e-6)
    return x[:, 1 + reg.shape[1]:]


# --------------------------------------------------------------------------
# Aggregator (sailrecon/models/aggregator.py)
# --------------------------------------------------------------------------

def build_allow_block(L: int, la: Sequence[int], lb: Sequence[int]) -> Tensor:
    """aggregator.py:832-847 (True = attend)."""
    allow = torch.zeros(L, L, dtype=torch.bool)
    ia = torch.tensor(list(la))
    allow[ia[:, None], ia[None, :]] = True
    if len(lb) > 0:
        ib = torch.tensor(list(lb))
        allow[ib[:, None], ia[None, :]] = True
        allow[ib, ib] = True
    return allow


def reloc_mask(S: int, Na: int, Nq: int, P: int, psi: int, rank: int) -> Tensor:
    """The global_reloc block's dense boolean mask (True = attend), aggregator.py:302-311."""
    allow = build_allow_block(S, list(range(Na)), [i + Na for i in range(Nq)])
    full = allow.repeat_interleave(P, 0).repeat_interleave(P, 1)
    cut = (P - psi - rank) * Na
    return full[cut:, cut:][None, None]


def draw_subsample_indices(generator: torch.Generator, depth: int, batch: int, n_anchor: int,
                           n_patch: int, rank: int) -> Tensor:
    """Replay of random_select_features' draws, aggregator.py:339,351-357,617-621.

    Order: layer -> batch -> anchor frame; each draw ``randperm(n_patch)[:rank]``.
    Returns int64 [depth, batch, n_anchor, rank].
    """
    out = torch.empty(depth, batch, n_anchor, rank, dtype=torch.long)
    for l in range(depth):
        for b in range(batch):
            for a in range(n_anchor):
                out[l, b, a] = torch.randperm(n_patch, generator=generator)[:rank]
    return out


class AggCfg:
    def __init__(self, patch=14, embed_dim=1024, depth=24, heads=16, dino_depth=24, dino_heads=16,
                 n_register=4, rope_base=100.0, inter_idx=(4, 11, 17, 23)):
        self.patch, self.C, self.depth, self.heads = patch, embed_dim, depth, heads
        self.dino_depth, self.dino_heads = dino_depth, dino_heads
        self.n_register, self.rope_base, self.inter_idx = n_register, rope_base, tuple(inter_idx)


def aggregator_forward(sd: SD, cfg: AggCfg, images: Tensor, no_reloc: List[int], reloc: List[int],
                       fix_rank: int, sub_idx: Tensor, pre: str = "aggregator.") -> Tuple[Dict[int, Tensor], int, Tensor]:
    """Aggregator.forward, aggregator.py:242-433, with explicit subsample indices.

    ``sub_idx``: int64 [depth, B, Na, rank] patch indices (see draw_subsample_indices).
    """
    B, S, _, H, W = images.shape
    Na, Nq = len(no_reloc), len(reloc)
    C = cfg.C
    psi = 1 + cfg.n_register
    mean = torch.tensor(RESNET_MEAN).view(1, 1, 3, 1, 1)
    std = torch.tensor(RESNET_STD).view(1, 1, 3, 1, 1)
    imgs = ((images - mean) / std).reshape(B * S, 3, H, W)  # :267-270
    patches = dino_forward(sd, pre + "patch_embed.", imgs, cfg.patch, cfg.dino_depth, cfg.dino_heads)
    n_patch = patches.shape[1]
    rank = min(fix_rank, n_patch)  # :277-278

    # special tokens, :287-299 + slice_expand_and_flatten :806-829
    def expand_special(t: Tensor) -> Tensor:
        first = t[:, 0:1].expand(B, 1, *t.shape[2:])
        rest = t[:, 1:].expand(B, S - 1, *t.shape[2:])
        return torch.cat([first, rest], dim=1).clone()

    cam = expand_special(sd[pre + "camera_token"])
    reg = expand_special(sd[pre + "register_token"])
    cam[:, reloc] = sd[pre + "camera_token_reloc"][:, 0:1].expand(B, Nq, *cam.shape[2:])
    reg[:, reloc] = sd[pre + "register_token_reloc"][:, 0:1].expand(B, Nq, *reg.shape[2:])
    tokens = torch.cat([cam.view(B * S, 1, C), reg.view(B * S, cfg.n_register, C), patches], dim=1)
    P = tokens.shape[1]
    P_prime = min(rank + psi, P)

    mask = reloc_mask(S, Na, Nq, P, psi, rank)

    # positions, :313-328 + PositionGetter rope.py:40-66
    hp, wp = H // cfg.patch, W // cfg.patch
    yy, xx = torch.meshgrid(torch.arange(hp), torch.arange(wp), indexing="ij")
    grid = torch.stack([yy.reshape(-1), xx.reshape(-1)], dim=-1) + 1
    pos = torch.cat([torch.zeros(psi, 2, dtype=torch.long), grid], dim=0)[None].expand(B * S, P, 2).contiguous()

    out: Dict[int, Tensor] = {}
    cam_last = None
    for layer in range(cfg.depth):  # :339
        tokens = block(sd, f"{pre}frame_blocks.{layer}.", tokens, cfg.heads, 1e-5, pos=pos,
                       qk_norm=True, rope_base=cfg.rope_base)  # :643-670
        frame_out = tokens.view(B, S, P, C)
        # select_scene_repe_for_reloc / random_select_features, :580-626
        anc = frame_out[:, no_reloc]
        anc_pos = pos.view(B, S, P, 2)[:, no_reloc]
        sel = sub_idx[layer][..., :rank] + psi  # token index of selected patches
        g_tok = torch.gather(anc, 2, sel[..., None].expand(B, Na, rank, C))
        g_pos = torch.gather(anc_pos, 2, sel[..., None].expand(B, Na, rank, 2))
        sub = torch.cat([anc[:, :, :psi], g_tok], dim=2).reshape(B, Na * P_prime, C)
        sub_pos = torch.cat([anc_pos[:, :, :psi], g_pos], dim=2).reshape(B, Na * P_prime, 2)
        # global_reloc block over [anchor subsample ; query frames] with mask, :672-741
        q_tok = frame_out[:, reloc].reshape(B, Nq * P, C)
        q_pos = pos.view(B, S, P, 2)[:, reloc].reshape(B, Nq * P, 2)
        seq = torch.cat([sub, q_tok], dim=1)
        seq = block(sd, f"{pre}global_reloc_blocks.{layer}.", seq, cfg.heads, 1e-5,
                    pos=torch.cat([sub_pos, q_pos], dim=1), mask=mask, qk_norm=True,
                    rope_base=cfg.rope_base)
        reloc_out = seq[:, Na * P_prime:]
        # global block over all anchor tokens, :743-769
        g = frame_out[:, no_reloc].reshape(B, Na * P, C)
        g = block(sd, f"{pre}global_blocks.{layer}.", g, cfg.heads, 1e-5,
                  pos=pos.view(B, S, P, 2)[:, no_reloc].reshape(B, Na * P, 2), qk_norm=True,
                  rope_base=cfg.rope_base)
        # reassembly, :393-399
        new = torch.ones(B, S, P, C, dtype=tokens.dtype)
        new[:, no_reloc] = g.view(B, Na, P, C)
        new[:, reloc] = reloc_out.view(B, Nq, P, C)
        # intermediates, :403-423
        if layer in cfg.inter_idx and Nq > 0:
            out[layer] = torch.cat([frame_out[:, reloc], reloc_out.view(B, Nq, P, C)], dim=-1)
        if layer == cfg.depth - 1:
            cam_last = torch.cat([frame_out[:, no_reloc][:, :, 0], g.view(B, Na, P, C)[:, :, 0]], dim=-1).clone()
        tokens = new.view(B * S, P, C)
    if Nq > 0:
        out[-1] = out[cfg.depth - 1]
    return out, psi, cam_last


# --------------------------------------------------------------------------
# Camera head (sailrecon/heads/camera_head.py, head_act.py)
# --------------------------------------------------------------------------

def build_lr_mask(S: int, no_reloc: Sequence[int]) -> Tensor:
    """camera_head.py:197-228 (True = MASKED)."""
    r_idx = torch.tensor([i for i in range(S) if i not in no_reloc], dtype=torch.long)
    l_idx = torch.as_tensor(list(no_reloc), dtype=torch.long).unique(sorted=True)
    m = torch.zeros(S, S, dtype=torch.bool)
    if l_idx.numel() and r_idx.numel():
        m[l_idx[:, None], r_idx[None, :]] = True
    if r_idx.numel() > 1:
        m[r_idx[:, None], r_idx[None, :]] = True
        m[r_idx, r_idx] = False
    return m[None, None]


def activate_pose(p: Tensor) -> Tensor:
    """activate_pose(trans linear, quat linear, fl relu), head_act.py:12-60."""
    return torch.cat([p[..., :3], p[..., 3:7], F.relu(p[..., 7:])], dim=-1)


def camera_head_forward(sd: SD, feats_last: Tensor, cam_last: Tensor, heads: int = 16, trunk_depth: int = 4,
                        iters: int = 4, pre: str = "camera_head.") -> List[Tensor]:
    """CameraHead.forward + trunk_fn, camera_head.py:85-186 (fp32)."""
    na = cam_last.shape[1]
    tok = torch.cat([cam_last, feats_last[:, :, 0]], dim=1)  # :103-109
    tok = layer_norm(tok, sd[pre + "token_norm.weight"], sd[pre + "token_norm.bias"], 1e-5)
    B, S, C = tok.shape
    attend = ~build_lr_mask(S, list(range(na)))  # :112-116,165
    pred = None
    outs = []
    for _ in range(iters):
        if pred is not None:  # :148-150 detach the previous prediction (no backprop through time)
            pred = pred.detach()
        inp = sd[pre + "empty_pose_tokens"].expand(B, S, -1) if pred is None else pred
        emb = F.linear(inp, sd[pre + "embed_pose.weight"], sd[pre + "embed_pose.bias"])
        mod = F.linear(F.silu(emb), sd[pre + "poseLN_modulation.1.weight"], sd[pre + "poseLN_modulation.1.bias"])
        shift, scale, gate = mod.chunk(3, dim=-1)
        x = gate * (layer_norm(tok, None, None, 1e-6) * (1 + scale) + shift) + tok  # :158-161
        for i in range(trunk_depth):
            x = block(sd, f"{pre}trunk.{i}.", x, heads, 1e-5, mask=attend)
        delta = mlp(sd, pre + "pose_branch.",
                    layer_norm(x, sd[pre + "trunk_norm.weight"], sd[pre + "trunk_norm.bias"], 1e-5))
        pred = delta if pred is None else pred + delta
        outs.append(activate_pose(pred))
    return [o[:, na:] for o in outs]


# --------------------------------------------------------------------------
# Pose decode (sailrecon/utils/pose_enc.py, rotation.py)
# --------------------------------------------------------------------------

def quat_to_mat(q: Tensor) -> Tensor:
    """rotation.py:14-44 (xyzw, scalar last)."""
    i, j, k, r = torch.unbind(q, -1)
    two_s = 2.0 / (q * q).sum(-1)
    o = torch.stack((1 - two_s * (j * j + k * k), two_s * (i * j - k * r), two_s * (i * k + j * r),
                     two_s * (i * j + k * r), 1 - two_s * (i * i + k * k), two_s * (j * k - i * r),
                     two_s * (i * k - j * r), two_s * (j * k + i * r), 1 - two_s * (i * i + j * j)), -1)
    return o.reshape(q.shape[:-1] + (3, 3))


def pose_encoding_to_extri_intri(enc: Tensor, hw: Tuple[int, int]) -> Tuple[Tensor, Tensor]:
    """pose_enc.py:68-135."""
    T, quat, fov_h, fov_w = enc[..., :3], enc[..., 3:7], enc[..., 7], enc[..., 8]
    ext = torch.cat([quat_to_mat(quat), T[..., None]], dim=-1)
    H, W = hw
    fy = (H / 2.0) / torch.tan(fov_h / 2.0)
    fx = (W / 2.0) / torch.tan(fov_w / 2.0)
    intr = torch.zeros(enc.shape[:2] + (3, 3))
    intr[..., 0, 0] = fx
    intr[..., 1, 1] = fy
    intr[..., 0, 2] = W / 2
    intr[..., 1, 2] = H / 2
    intr[..., 2, 2] = 1.0
    return ext, intr


# --------------------------------------------------------------------------
# end-to-end hot path (SailRecon.forward minus DPT heads), sail_recon.py:70-124
# --------------------------------------------------------------------------

def hot_path_forward(sd: SD, cfg: AggCfg, images: Tensor, no_reloc: List[int], reloc: List[int],
                     fix_rank: int, sub_idx: Tensor, cam_heads: int = 16, cam_depth: int = 4) -> Dict[str, object]:
    with torch.no_grad():
        feats, psi, cam_last = aggregator_forward(sd, cfg, images, no_reloc, reloc, fix_rank, sub_idx)
        poses = camera_head_forward(sd, feats[-1], cam_last, heads=cam_heads, trunk_depth=cam_depth)
        ext, intr = pose_encoding_to_extri_intri(poses[-1], (images.shape[-2], images.shape[-1]))
    return {"feats": feats, "patch_start_idx": psi, "cam_token_last_layer": cam_last,
            "pose_enc_list": poses, "extrinsic": ext, "intrinsic": intr}


# --------------------------------------------------------------------------
# DPT point / depth heads (sailrecon/heads/dpt_head.py, utils.py, head_act.py) and
# the depth unprojection (sailrecon/utils/geometry.py) — SURVEY §8(f) rank 1
# --------------------------------------------------------------------------

def _uv_pos_embed(h: int, w: int, c: int, aspect: float) -> Tensor:
    """[h, w, c] uv-grid sin/cos embedding (utils.py create_uv_grid + position_grid_to_embed):
    x half then y half, each [sin | cos] of pos * 100^(-i / (c/4)), evaluated in double."""
    diag = (aspect ** 2 + 1.0) ** 0.5
    sx, sy = aspect / diag, 1.0 / diag
    xs = torch.linspace(-sx * (w - 1) / w, sx * (w - 1) / w, steps=w, dtype=torch.float32)
    ys = torch.linspace(-sy * (h - 1) / h, sy * (h - 1) / h, steps=h, dtype=torch.float32)
    q = c // 4
    omega = 1.0 / 100.0 ** (torch.arange(q, dtype=torch.float64) / q)

    def one(pos):  # [n] -> [n, c/2]
        arg = pos.double()[:, None] * omega[None]
        return torch.cat([arg.sin(), arg.cos()], 1).float()

    ex = one(xs)[None, :, :].expand(h, w, c // 2)
    ey = one(ys)[:, None, :].expand(h, w, c // 2)
    return torch.cat([ex, ey], -1)


def _add_pos(x: Tensor, aspect: float, ratio: float = 0.1) -> Tensor:  # x NCHW
    pe = _uv_pos_embed(x.shape[2], x.shape[3], x.shape[1], aspect) * ratio
    return x + pe.permute(2, 0, 1)[None]


def _conv(sd: SD, pre: str, x: Tensor, stride: int = 1, pad: Optional[int] = None) -> Tensor:
    w = sd[pre + ".weight"]
    if pad is None:
        pad = w.shape[-1] // 2
    return F.conv2d(x, w, sd.get(pre + ".bias"), stride=stride, padding=pad)


def _rcu(sd: SD, pre: str, x: Tensor) -> Tensor:  # dpt_head.py:470-487
    # the reference's activation is nn.ReLU(inplace=True) applied to the unit's own input, so
    # the skip connection adds relu(x), not x (dpt_head.py:377-380, 470-487)
    x = F.relu(x)
    out = _conv(sd, pre + ".conv1", x)
    out = _conv(sd, pre + ".conv2", F.relu(out))
    return out + x


def _fusion(sd: SD, pre: str, x0: Tensor, x1: Optional[Tensor], size) -> Tensor:  # dpt_head.py:540-565
    out = x0
    if x1 is not None and (pre + ".resConfUnit1.conv1.weight") in sd:
        out = out + _rcu(sd, pre + ".resConfUnit1", x1)
    out = _rcu(sd, pre + ".resConfUnit2", out)
    if size is None:
        size = (int(out.shape[2] * 2), int(out.shape[3] * 2))
    out = F.interpolate(out, size=size, mode="bilinear", align_corners=True)
    return _conv(sd, pre + ".out_conv", out)


def dpt_forward(sd: SD, pre: str, tokens: Dict[int, Tensor], images: Tensor, patch_start: int,
                layers: Sequence[int] = (4, 11, 17, 23), activation: str = "inv_log",
                conf_activation: str = "expp1", patch: int = 14, feature_only: bool = False):
    """DPTHead.forward (dpt_head.py:151-298) for all frames at once; returns (preds, conf), or with
    feature_only the fused feature map [B, S, features, H, W] (dpt_head.py:123-126,286-287)."""
    B, S, _, H, W = images.shape
    ph, pw = H // patch, W // patch
    aspect = W / H
    feats = []
    for i, l in enumerate(layers):
        x = tokens[l][:, :, patch_start:].reshape(B * S, ph * pw, -1)
        x = layer_norm(x, sd[pre + "norm.weight"], sd[pre + "norm.bias"], 1e-5)
        x = x.permute(0, 2, 1).reshape(B * S, -1, ph, pw)
        x = _conv(sd, pre + f"projects.{i}", x)
        x = _add_pos(x, aspect)
        rp = pre + f"resize_layers.{i}"
        if i in (0, 1):
            x = F.conv_transpose2d(x, sd[rp + ".weight"], sd[rp + ".bias"], stride=4 if i == 0 else 2)
        elif i == 3:
            x = _conv(sd, rp, x, stride=2, pad=1)
        feats.append(x)
    rn = [_conv(sd, pre + f"scratch.layer{i + 1}_rn", f) for i, f in enumerate(feats)]
    out = _fusion(sd, pre + "scratch.refinenet4", rn[3], None, rn[2].shape[2:])
    out = _fusion(sd, pre + "scratch.refinenet3", out, rn[2], rn[1].shape[2:])
    out = _fusion(sd, pre + "scratch.refinenet2", out, rn[1], rn[0].shape[2:])
    out = _fusion(sd, pre + "scratch.refinenet1", out, rn[0], None)
    out = _conv(sd, pre + "scratch.output_conv1", out)
    out = F.interpolate(out, size=(ph * patch, pw * patch), mode="bilinear", align_corners=True)
    out = _add_pos(out, aspect)
    if feature_only:
        return out.view(B, S, *out.shape[1:])
    out = F.relu(_conv(sd, pre + "scratch.output_conv2.0", out))
    out = _conv(sd, pre + "scratch.output_conv2.2", out)
    fmap = out.permute(0, 2, 3, 1)
    xyz, cf = fmap[..., :-1], fmap[..., -1]
    if activation == "inv_log":  # head_act.py:117-127
        pts = torch.sign(xyz) * torch.expm1(xyz.abs())
    elif activation == "exp":
        pts = xyz.exp()
    else:
        raise ValueError(activation)
    conf = 1 + cf.exp() if conf_activation == "expp1" else cf.exp()
    return pts.reshape(B, S, H, W, -1), conf.reshape(B, S, H, W)


def unproject_depth(depth: Tensor, extr: Tensor, intr: Tensor) -> Tensor:
    """geometry.py:19-130 in float64: depth [S,H,W(,1)] -> world points [S,H,W,3]."""
    if depth.dim() == 4:
        depth = depth[..., 0]
    S, H, W = depth.shape
    v, u = torch.meshgrid(torch.arange(H, dtype=torch.float64), torch.arange(W, dtype=torch.float64), indexing="ij")
    out = []
    for s in range(S):
        K, E, d = intr[s].double(), extr[s].double(), depth[s].double()
        cam = torch.stack([(u - K[0, 2]) * d / K[0, 0], (v - K[1, 2]) * d / K[1, 1], d], -1)
        R, t = E[:, :3], E[:, 3]
        out.append(cam @ R + (-(R.T @ t)))  # R_c2w = R^T: cam @ R_c2w^T = cam @ R
    return torch.stack(out)


# --------------------------------------------------------------------------
# Input formation (train/utils/io.py:75-195 ImagePreprocessor; datasets/imc2021.py:260-301):
# pad to square (zeros, centred), PIL BICUBIC resize to target, ToTensor / uint16 depth / 1000,
# K <-> K' matrices — SURVEY §8(f) rank 2.  PIL's resample (Pillow Resample.c) restated.
# --------------------------------------------------------------------------

PIL_PRECISION_BITS = 32 - 8 - 2


def _pil_bicubic(x: float, a: float = -0.5) -> float:
    x = abs(x)
    if x < 1.0:
        return ((a + 2.0) * x - (a + 3.0)) * x * x + 1
    if x < 2.0:
        return (((x - 5) * x + 8) * x - 4) * a
    return 0.0


def pil_coeffs(in_size: int, out_size: int):
    """Per output pixel: (first input index, normalised double weights) of PIL's antialiased
    bicubic filter (support 2 * max(scale, 1), centre (i + 0.5) * scale)."""
    scale = in_size / out_size
    fs = max(scale, 1.0)
    support, ss = 2.0 * fs, 1.0 / fs
    out = []
    for xx in range(out_size):
        c = (xx + 0.5) * scale
        xmin = max(int(c - support + 0.5), 0)
        xmax = min(int(c + support + 0.5), in_size) - xmin
        k = [_pil_bicubic((x + xmin - c + 0.5) * ss) for x in range(xmax)]
        ww = sum(k)
        out.append((xmin, [w / ww if ww != 0.0 else w for w in k]))
    return out


def pil_fixed(k):
    """8-bit modes: weights as PRECISION_BITS fixed point (rounded away from zero)."""
    s = 1 << PIL_PRECISION_BITS
    return [int(-0.5 + w * s) if w < 0 else int(0.5 + w * s) for w in k]


def pil_resize_u8(img, target: int):
    """uint8 [h, w, c] -> [target, target, c]: horizontal then vertical integer pass, each
    rounded (+half), shifted and clipped to 0..255."""
    import numpy as np
    h, w, c = img.shape
    P = PIL_PRECISION_BITS

    def run(src, coeffs, axis):
        n = len(coeffs)
        shape = list(src.shape)
        shape[axis] = n
        out = np.zeros(shape, np.int64)
        for i, (xmin, k) in enumerate(coeffs):
            kk = np.array(pil_fixed(k), np.int64)
            seg = np.take(src, range(xmin, xmin + len(kk)), axis=axis).astype(np.int64)
            acc = np.tensordot(seg, kk, axes=([axis], [0])) + (1 << (P - 1))
            idx = [slice(None)] * src.ndim
            idx[axis] = i
            out[tuple(idx)] = np.clip(acc >> P, 0, 255)
        return out

    tmp = run(img, pil_coeffs(w, target), 1)
    return run(tmp, pil_coeffs(h, target), 0).astype(np.uint8)


def pil_resize_u16(img, target: int):
    """'I;16' [h, w] -> [target, target]: double accumulation in tap order, round half away from
    zero, stored as CLIP8(v % 256) | CLIP8(v >> 8) << 8 after each pass (Pillow's 16-bit path)."""
    import numpy as np
    h, w = img.shape

    def store(v):
        vi = np.where(v >= 0, np.trunc(v + 0.5), np.trunc(v - 0.5)).astype(np.int64)
        return np.clip(np.fmod(vi, 256), 0, 255) + (np.clip(vi >> 8, 0, 255) << 8)

    tmp = np.zeros((h, target), np.int64)
    for xx, (xmin, k) in enumerate(pil_coeffs(w, target)):
        acc = np.zeros(h)
        for j, kw in enumerate(k):
            acc = acc + img[:, xmin + j].astype(np.float64) * kw
        tmp[:, xx] = store(acc)
    out = np.zeros((target, target), np.int64)
    for yy, (ymin, k) in enumerate(pil_coeffs(h, target)):
        acc = np.zeros(target)
        for j, kw in enumerate(k):
            acc = acc + tmp[ymin + j].astype(np.float64) * kw
        out[yy] = store(acc)
    return out.astype(np.uint16)


def preprocess_image(img, target: int = 518, is_depth: bool = False):
    """ImagePreprocessor.process_image_with_matrices (io.py:75-195) on a uint8 [h, w, 3] RGB or
    uint16 [h, w] depth array: (tensor [1, C, T, T] fp32, K_to_K_prime, K_prime_to_K)."""
    import numpy as np
    h, w = img.shape[:2]
    m = max(h, w)
    pl, pt = (m - w) // 2, (m - h) // 2
    sq = np.zeros((m, m) + img.shape[2:], img.dtype)
    sq[pt:pt + h, pl:pl + w] = img
    if is_depth:
        r = pil_resize_u16(sq, target).astype(np.float32) / 1000
        t = torch.from_numpy(r)[None]
    else:
        r = pil_resize_u8(sq, target)
        t = torch.from_numpy(r).permute(2, 0, 1).float().div(255)
    s = target / m
    k2kp = torch.tensor([[s, 0.0, pl * s], [0.0, s, pt * s], [0.0, 0.0, 1.0]], dtype=torch.float32)
    kp2k = torch.tensor([[1.0 / s, 0.0, -(pl * s) / s], [0.0, 1.0 / s, -(pt * s) / s], [0.0, 0.0, 1.0]],
                        dtype=torch.float32)
    return t[None], k2kp, kp2k


def reverse_transform_tensor(processed: Tensor, kp2k: Tensor, target: int, is_depth: bool = False) -> Tensor:
    """ImagePreprocessor.reverse_transform_tensor (train/utils/io.py:197-259) restated line by line
    with the same torch calls (the reference module itself does not import here: cv2 / torchvision
    are absent): scale and padding read back from K_prime_to_K, F.interpolate to max_side
    (bicubic for RGB, bilinear for depth, align_corners=False), crop of the padding."""
    import torch.nn.functional as F
    scale_x = 1.0 / kp2k[0, 0].item()
    scale_y = 1.0 / kp2k[1, 1].item()
    offset_x = -kp2k[0, 2].item() * scale_x
    offset_y = -kp2k[1, 2].item() * scale_y
    max_side = int(target / scale_x)
    pad_left = int(offset_x / scale_x)
    pad_top = int(offset_y / scale_y)
    r = F.interpolate(processed.unsqueeze(0), size=(max_side, max_side),
                      mode="bicubic" if not is_depth else "bilinear", align_corners=False).squeeze(0)
    w, h = max_side - 2 * pad_left, max_side - 2 * pad_top
    return r[:, pad_top:pad_top + h, pad_left:pad_left + w]


# --------------------------------------------------------------------------
# Self-supervised training loss: compute_loss (train/train_imc.py:141-246)
# with CDFLossIndexPytorch (train/losses/cdf_loss.py:19-242) and the projective geometry of
# train/utils/geometry.py:89-303.  Pinned by tests/golden/g8_loss.npz (reference modules).
# --------------------------------------------------------------------------

def cdf_smooth_kernel(bin_width: float, gradient_smooth: float) -> Tensor:
    """cdf_loss.py:62-84: Gaussian smoothing taps (identity [1.0] when smoothing is off)."""
    if gradient_smooth <= 0:
        return torch.ones(1)
    r = max(1, int(gradient_smooth / bin_width))
    idx = torch.arange(2 * r + 1, dtype=torch.float32) - r
    sigma = gradient_smooth / bin_width
    g = torch.exp(-0.5 * (idx / sigma) ** 2)
    return g / torch.sum(g)


def _reflect_conv(x: Tensor, taps: Tensor) -> Tensor:
    """Conv1d(padding=len//2, padding_mode='reflect') over the last dim (cross-correlation)."""
    r = taps.numel() // 2
    if r == 0:
        return x * taps[0]
    xp = F.pad(x[:, None], (r, r), mode="reflect")[:, 0]
    return sum(taps[k] * xp[:, k:k + x.shape[1]] for k in range(taps.numel()))


def cdf_loss_values(res: Tensor, w: Tensor, node_src: Tensor, node_dst: Tensor, n_nodes: int,
                    min_val: float = 0.0, max_val: float = 15.0, num_bins: int = 250,
                    gradient_smooth: float = 0.05) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    """CDFLossIndexPytorch.forward's values and gradients (cdf_loss.py:88-242):
    (cdf_src, grad_src, cdf_dst, grad_dst), each [pairs, points]."""
    P, K = res.shape
    bw = (max_val - min_val) / num_bins
    b = ((res - min_val) / bw).long()                                    # :136-139 histogram bin
    ok = ((b >= 0) & (b < num_bins)).float()
    b = b.clamp(0, num_bins - 1)
    hist = torch.zeros(n_nodes * num_bins)
    tot = torch.zeros(n_nodes)
    ns = node_src.long()[:, None].expand(P, K).reshape(-1)
    nd = node_dst.long()[:, None].expand(P, K).reshape(-1)
    hist.index_add_(0, ns * num_bins + b.reshape(-1), (w * ok).reshape(-1))
    hist.index_add_(0, nd * num_bins + b.reshape(-1), (w * ok).reshape(-1))
    tot.index_add_(0, ns, w.reshape(-1))
    tot.index_add_(0, nd, w.reshape(-1))
    pmf = hist.view(n_nodes, num_bins) / (tot[:, None] + 1e-10)          # :177
    cdf = torch.cumsum(pmf, 1)
    sobel = torch.tensor([-1.0, 0.0, 1.0]) / (2.0 * bw)                  # :59-60
    pdf = _reflect_conv(_reflect_conv(cdf, sobel), cdf_smooth_kernel(bw, gradient_smooth))
    bl = ((res - min_val) / bw + 0.5).long()                              # :207-210 lookup bin
    valid = (bl >= 0) & (bl < num_bins) & (w > 0)
    bl = bl.clamp(0, num_bins - 1)
    gs = node_src.long()[:, None] * num_bins + bl
    gd = node_dst.long()[:, None] * num_bins + bl
    fc, fp = cdf.reshape(-1), pdf.reshape(-1)
    cs, cd = fc[gs], fc[gd]
    two = torch.full_like(cs, 2.0)
    return (torch.where(valid, cs, two), torch.where(valid, fp[gs] * w, torch.zeros_like(cs)),
            torch.where(valid, cd, two), torch.where(valid, fp[gd] * w, torch.zeros_like(cs)))


def _cdf_straight_through(res: Tensor, w: Tensor, *cdf_args) -> Tuple[Tensor, Tensor]:
    """CDFLossTorchWrapper (cdf_loss.py:6-16): value = CDF lookup, d/dres = pdf * w."""
    cs, gs, cd, gd = cdf_loss_values(res.detach(), w, *cdf_args)
    return cs + (res - res.detach()) * gs, cd + (res - res.detach()) * gd


def imc_loss(enc: Tensor, hw: Tuple[int, int], kp2k: Tensor, shared_focal: bool, src_idx: Tensor, dst_idx: Tensor,
             src_coords: Tensor, dst_coords: Tensor, src_depth: Tensor, dst_depth: Tensor, node_src: Tensor,
             node_dst: Tensor, n_nodes: int, min_val: float = 0.0, max_val: float = 15.0, num_bins: int = 250,
             gradient_smooth: float = 0.05) -> Tensor:
    """compute_loss (train_imc.py:141-246) for pose encodings enc [N, 9] (differentiable)."""
    ext, intr = pose_encoding_to_extri_intri(enc[None], hw)
    K = torch.bmm(kp2k, intr[0])                                           # :166 K' -> K
    if shared_focal:                                                      # :169-174
        K = K.mean(0, keepdim=True).repeat(K.shape[0], 1, 1)
    pad = torch.tensor([0.0, 0.0, 0.0, 1.0])

    def pad44(e):                                                         # geometry.py pad_poses
        return torch.cat([e, pad.expand(e.shape[0], 1, 4)], 1)
    Es, Ed = pad44(ext[0][src_idx.long()]), pad44(ext[0][dst_idx.long()])
    rel = torch.bmm(Ed, torch.inverse(Es))                                # compute_relative_pose
    Ks, Kd = K[src_idx.long()], K[dst_idx.long()]
    h = torch.cat([src_coords, torch.ones_like(src_coords[..., :1])], -1)
    X = torch.bmm(torch.inverse(Ks), h.transpose(1, 2)).transpose(1, 2) * src_depth[..., None]
    Y = torch.bmm(rel, torch.cat([X, torch.ones_like(X[..., :1])], -1).transpose(1, 2)).transpose(1, 2)[..., :3]
    p = torch.bmm(Kd, Y.transpose(1, 2)).transpose(1, 2)
    pred = p[..., :2] / (p[..., 2:] + 1e-6)                               # from_homogeneous
    pred2 = p[..., :2] / (dst_depth[..., None] + 1e-6)                    # approximation variant
    w = torch.ones_like(src_depth)                                        # valid masks: all ones
    args = (node_src, node_dst, n_nodes, min_val, max_val, num_bins, gradient_smooth)
    total = 0.0
    for pr in (pred, pred2):
        res = torch.log1p(torch.norm(pr - dst_coords, dim=-1))            # :212-238
        a, b = _cdf_straight_through(res, w, *args)
        total = total + (a.mean() + b.mean()) / 2.0
    return total / 2.0
