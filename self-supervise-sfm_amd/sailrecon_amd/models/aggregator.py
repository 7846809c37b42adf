"""Aggregator — MI355X-native re-design of sailrecon/models/aggregator.py.

Same constructor arguments, parameter names and ``forward(images, no_reloc_list,
reloc_list, fix_rank)`` contract as the reference (aggregator.py:62-85, 242-433).

Layout (SURVEY §7 design stance):
  * ONE fp32 residual buffer x [B*S*P, C] for the whole forward; frames are ordered
    internally as [anchors (no_reloc_list order) ; queries (reloc_list order)] per
    batch item, so the global stack is the contiguous anchor slice and the reloc
    stack the contiguous query slice — no torch.ones + scatter reassembly
    (aggregator.py:393-399) and no dense (S*P)^2 mask (aggregator.py:302-311);
  * every Block is the 7-launch HIP sequence of runtime.run_block;
  * the anchor subsample (aggregator.py:580-626) is a row map: its LayerNorm reads
    the selected rows directly and only their K/V are projected (their query rows
    are discarded by the reference, aggregator.py:737);
  * global_reloc attention = segment 0 (shared anchor subsample K/V) + segment 1
    (own frame), exactly the reference mask's allowed set;
  * subsample draws replay the reference generator order (layer -> batch -> anchor,
    ``randperm(n_patch, generator)[:rank]``) on the host while the GPU runs DINO.
"""

from __future__ import annotations

import logging
from typing import Dict, List, Optional, Tuple, Union

import numpy as np
import torch
import torch.nn as nn

from .. import _lib, ops, runtime
from ..layers import PatchEmbed
from ..layers.block import Block
from ..layers.rope import PositionGetter, RotaryPositionEmbedding2D
from ..layers.vision_transformer import vit_base, vit_giant2, vit_large, vit_small

logger = logging.getLogger(__name__)

_RESNET_MEAN = [0.485, 0.456, 0.406]
_RESNET_STD = [0.229, 0.224, 0.225]


class Aggregator(nn.Module):
    def __init__(self, img_size=518, patch_size=14, embed_dim=1024, depth=24, num_heads=16, mlp_ratio=4.0,
                 num_register_tokens=4, block_fn=Block, qkv_bias=True, proj_bias=True, ffn_bias=True,
                 patch_embed="dinov2_vitl14_reg", aa_order=["frame", "global"], aa_block_size=1, qk_norm=True,
                 rope_freq=100, init_values=0.01, intermediate_layer_idx=[4, 11, 17, 23], min_rank: int = 150,
                 kv_cache: bool = False):
        super().__init__()
        if list(aa_order) != ["frame", "global"] or aa_block_size != 1:
            raise NotImplementedError("the SailRecon hot path uses aa_order=['frame','global'], aa_block_size=1")
        self.__build_patch_embed__(patch_embed, img_size, patch_size, num_register_tokens, embed_dim=embed_dim)
        self.rope = RotaryPositionEmbedding2D(frequency=rope_freq) if rope_freq > 0 else None
        self.position_getter = PositionGetter() if self.rope is not None else None
        self.intermediate_layer_idx = intermediate_layer_idx

        def blocks(cache=False):
            return nn.ModuleList([block_fn(dim=embed_dim, num_heads=num_heads, mlp_ratio=mlp_ratio, qkv_bias=qkv_bias,
                                           proj_bias=proj_bias, ffn_bias=ffn_bias, init_values=init_values,
                                           qk_norm=qk_norm, rope=self.rope, kv_cache=cache) for _ in range(depth)])

        self.frame_blocks = blocks()
        self.global_blocks = blocks()
        self.global_reloc_blocks = blocks(kv_cache)
        self.depth = depth
        self.aa_order = aa_order
        self.patch_size = patch_size
        self.aa_block_size = aa_block_size
        self.aa_block_num = depth // aa_block_size
        self.embed_dim = embed_dim
        self.num_heads = num_heads
        self.camera_token = nn.Parameter(torch.randn(1, 2, 1, embed_dim))
        self.register_token = nn.Parameter(torch.randn(1, 2, num_register_tokens, embed_dim))
        self.camera_token_reloc = nn.Parameter(torch.randn(1, 1, 1, embed_dim))
        self.register_token_reloc = nn.Parameter(torch.randn(1, 1, num_register_tokens, embed_dim))
        self.patch_start_idx = 1 + num_register_tokens
        self.num_register_tokens = num_register_tokens
        for p in (self.camera_token, self.register_token, self.camera_token_reloc, self.register_token_reloc):
            nn.init.normal_(p, std=1e-6)
        for name, value in (("_resnet_mean", _RESNET_MEAN), ("_resnet_std", _RESNET_STD)):
            self.register_buffer(name, torch.FloatTensor(value).view(1, 1, 3, 1, 1), persistent=False)
        self.min_rank = min_rank
        self.use_reentrant = False
        self.generator = self._generate_per_rank_generator()
        # None: follow autocast (bf16 under torch.autocast, exact fp32 otherwise)
        self.compute_dtype: Optional[torch.dtype] = None
        self._ws = runtime.Workspace()
        self._packed: Dict[Tuple[str, torch.dtype], object] = {}
        self.last_subsample_indices: Optional[torch.Tensor] = None

    # ------------------------------------------------------------------ construction
    def __build_patch_embed__(self, patch_embed, img_size, patch_size, num_register_tokens,
                              interpolate_antialias=True, interpolate_offset=0.0, block_chunks=0, init_values=1.0,
                              embed_dim=1024):
        """aggregator.py:196-240."""
        if "conv" in patch_embed:
            self.patch_embed = PatchEmbed(img_size=img_size, patch_size=patch_size, in_chans=3, embed_dim=embed_dim)
        else:
            vit_models = {"dinov2_vitl14_reg": vit_large, "dinov2_vitb14_reg": vit_base,
                          "dinov2_vits14_reg": vit_small, "dinov2_vitg2_reg": vit_giant2}
            self.patch_embed = vit_models[patch_embed](img_size=img_size, patch_size=patch_size,
                                                       num_register_tokens=num_register_tokens,
                                                       interpolate_antialias=interpolate_antialias,
                                                       interpolate_offset=interpolate_offset,
                                                       block_chunks=block_chunks, init_values=init_values)
            if hasattr(self.patch_embed, "mask_token"):
                self.patch_embed.mask_token.requires_grad_(False)

    def _generate_per_rank_generator(self):
        """aggregator.py:628-641.  Multi-GPU sharding (parallel.py) uses ONE draw
        sequence on every rank instead of per-rank seeds, so results do not depend on
        the world size (SURVEY §7 hard parts)."""
        seed = torch.randint(0, 2 ** 32, (1,)).item()
        rank = torch.distributed.get_rank() if torch.distributed.is_initialized() else 0
        g = torch.Generator()
        g.manual_seed(seed + rank)
        return g

    def invalidate_packed(self):
        """Call after changing parameters in place (load_state_dict does it automatically)."""
        self._packed.clear()
        for m in self.modules():
            if isinstance(m, Block):
                m.invalidate_packed()

    def _load_from_state_dict(self, *args, **kwargs):
        self.invalidate_packed()
        return super()._load_from_state_dict(*args, **kwargs)

    def _pack_misc(self, dtype: torch.dtype, kpad: int):
        key = ("misc", dtype, kpad)
        if key not in self._packed:
            pe = self.patch_embed
            conv = pe.patch_embed.proj if hasattr(pe, "blocks") else pe.proj
            C = conv.weight.shape[0]
            w = conv.weight.detach().reshape(C, -1).float()
            wp = torch.zeros(C, kpad, device=w.device, dtype=torch.float32)
            wp[:, : w.shape[1]] = w
            nreg = self.num_register_tokens
            table = torch.empty(3, 1 + nreg, C, device=w.device, dtype=torch.float32)
            table[0, 0] = self.camera_token[0, 0, 0]
            table[1, 0] = self.camera_token[0, 1, 0]
            table[2, 0] = self.camera_token_reloc[0, 0, 0]
            table[0, 1:] = self.register_token[0, 0]
            table[1, 1:] = self.register_token[0, 1]
            table[2, 1:] = self.register_token_reloc[0, 0]
            self._packed[key] = dict(w_patch=wp.to(dtype).contiguous(), b_patch=conv.bias.detach().float().contiguous(),
                                     special=table.detach().contiguous())
        return self._packed[key]

    # ------------------------------------------------------------------ subsample draws
    def draw_subsample(self, depth: int, B: int, na: int, n_patch: int, rank: int) -> np.ndarray:
        """Replays random_select_features' draws (aggregator.py:339,351-357,617-621):
        order layer -> batch -> anchor, ``randperm(n_patch, generator)[:rank]``."""
        out = np.empty((depth, B, na, rank), dtype=np.int64)
        for l in range(depth):
            for b in range(B):
                for a in range(na):
                    out[l, b, a] = torch.randperm(n_patch, generator=self.generator)[:rank].numpy()
        return out

    # ------------------------------------------------------------------ forward
    def forward(self, images: torch.Tensor, no_reloc_list: list, reloc_list: list,
                fix_rank: Union[int, None] = None) -> Tuple[Dict[int, torch.Tensor], int, torch.Tensor]:
        B, S, C_in, H, W = images.shape
        num_recon, num_reloc = len(no_reloc_list), len(reloc_list)
        self.num_recon = num_recon
        if C_in != 3:
            raise ValueError(f"Expected 3 input channels, got {C_in}")
        if not images.is_cuda:
            raise RuntimeError("sailrecon_amd Aggregator runs on the HIP path only (images must be on a ROCm device)")
        if sorted(list(no_reloc_list) + list(reloc_list)) != list(range(S)):
            raise ValueError("no_reloc_list and reloc_list must be disjoint and cover every frame "
                             f"(S={S}, got {list(no_reloc_list)} / {list(reloc_list)}); the reference's "
                             "block mask (aggregator.py:302-311) assumes the same")
        if num_recon == 0:
            raise ValueError("at least one anchor (no_reloc) frame is required")
        ps = self.patch_size
        assert H % ps == 0 and W % ps == 0, f"image size {H}x{W} is not a multiple of the patch size {ps}"
        dev = images.device
        dtype = runtime.compute_dtype(self.compute_dtype)
        C, nh = self.embed_dim, self.num_heads
        gh, gw = H // ps, W // ps
        n_patch = gh * gw
        psi = self.patch_start_idx
        P = n_patch + psi
        Na, Nq = num_recon, num_reloc
        F_ = B * S
        R = F_ * P
        ws = self._ws
        hidden = self.frame_blocks[0].mlp.fc1.out_features

        # ---- internal frame order: anchors then queries (per batch item)
        order = list(no_reloc_list) + list(reloc_list)
        imgs = images if order == list(range(S)) else images[:, order]
        imgs = imgs.reshape(F_, 3, H, W).float().contiguous()

        x = ws.get("x", R, C, torch.float32, dev)
        sc = runtime.scratch(ws, R, C, hidden, dtype, dev)

        # ---- patch embed (+ DINOv2 stack), vision_transformer.py:242-307
        kt = 64 if dtype == torch.bfloat16 else 32
        kpad = -(-3 * ps * ps // kt) * kt
        misc = self._pack_misc(dtype, kpad)
        cols = ws.get("im2col", F_ * n_patch, kpad, dtype, dev)
        ops.im2col_normalize(imgs, ps, cols, kpad)
        is_dino = hasattr(self.patch_embed, "blocks")
        if is_dino:
            dino = self.patch_embed
            pos_tab = dino.pos_embed_for(H, W)  # [1 + n_patch, C] fp32
            row_add = pos_tab[1:]
        else:
            row_add = ws.get("zeros_pos", n_patch, C, torch.float32, dev).zero_()
        ops.gemm(cols, misc["w_patch"], x, _lib.SR_EPI_PATCH, bias=misc["b_patch"], rows=F_ * n_patch,
                 patch=dict(seg_rows=n_patch, seg_stride=P, seg_offset=psi, row_add=row_add))
        if is_dino:
            nreg_d = dino.num_register_tokens
            if 1 + nreg_d != psi:
                raise NotImplementedError("DINO register count must equal the aggregator's")
            dtab = torch.cat([(dino.cls_token[0, 0] + pos_tab[0])[None], dino.register_tokens[0]], 0)
            dtab = dtab.detach().float().contiguous()[None]
            zero_t = ws.get("frame_type0", F_, 1, torch.int32, dev).zero_()
            ops.set_special_tokens(x, F_, P, dtab, zero_t)
            for blk in dino.blocks:
                pb = blk.packed(dtype)
                runtime.run_block(pb, x, 0, R, sc, runtime.frame_attend(pb, F_, P), None)
            ops.layernorm(x, dino.norm.weight, dino.norm.bias, dino.norm.eps, x)  # in place (row-local)

        # ---- aggregator special tokens, aggregator.py:287-299
        ftype = []
        for b in range(B):
            ftype += [0 if no_reloc_list[a] == 0 else 1 for a in range(Na)] + [2] * Nq
        ftype_t = torch.tensor(ftype, dtype=torch.int32).to(dev, non_blocking=True)
        ops.set_special_tokens(x, F_, P, misc["special"], ftype_t)

        # ---- subsample draws (host, overlaps the GPU work above), aggregator.py:277-285, 580-626
        if fix_rank is not None:
            self.rank = min(fix_rank, n_patch)
        else:
            lo, hi = min(self.min_rank, n_patch // 2), max(self.min_rank, n_patch // 2)
            self.rank = int(torch.randint(lo, hi, (1,), generator=self.generator).item())
        rank = self.rank
        Pp = min(rank + psi, P)
        idx = self.draw_subsample(self.depth, B, Na, n_patch, rank) if Nq > 0 else None
        if idx is not None:
            self.last_subsample_indices = torch.from_numpy(idx)
            base = (np.arange(B) * S * P)[None, :, None, None] + (np.arange(Na) * P)[None, None, :, None]
            sel = base + psi + idx                                       # [depth, B, Na, rank]
            spec = np.broadcast_to(base + np.arange(psi)[None, None, None, :], (self.depth, B, Na, psi))
            rowmap = np.concatenate([spec, sel], axis=-1).reshape(self.depth, B, Na * Pp).astype(np.int32)
            rowmap_t = torch.from_numpy(rowmap).pin_memory().to(dev, non_blocking=True)
        rope = self.rope.tables(C // nh, max(gh, gw) + 1, dev) if self.rope is not None else None
        posctx = dict(tokens_per_frame=P, patch_start=psi, grid_w=gw)

        # ---- outputs
        out_maps: Dict[int, torch.Tensor] = {}
        if Nq > 0:
            for l in self.intermediate_layer_idx:
                out_maps[l] = torch.empty(B, Nq, P, 2 * C, device=dev, dtype=torch.float32)
        cam_last = torch.empty(B, Na, 2 * C, device=dev, dtype=torch.float32)
        anchor_rows0 = torch.tensor([b * S * P + a * P for b in range(B) for a in range(Na)],
                                    dtype=torch.int32).to(dev, non_blocking=True)
        cam_flat = cam_last.view(B * Na, 2 * C)

        # ---- alternating layers, aggregator.py:339-423
        for l in range(self.depth):
            pb = self.frame_blocks[l].packed(dtype)
            runtime.run_block(pb, x, 0, R, sc, runtime.frame_attend(pb, F_, P),
                              runtime.qkv_params(pb, rope, pos_row_base=0, **posctx))
            if l in out_maps:  # frame half of the intermediate, :403-413
                om = out_maps[l]
                for b in range(B):
                    ops.copy_rows(om[b].view(Nq * P, 2 * C)[:, :C], x[b * S * P + Na * P:(b + 1) * S * P], Nq * P)
            if l == self.depth - 1:  # :414-423 frame half
                ops.copy_rows(cam_flat[:, :C], x, B * Na, rowmap=anchor_rows0)
            pr = self.global_reloc_blocks[l].packed(dtype)
            pg = self.global_blocks[l].packed(dtype)
            for b in range(B):
                a0, q0, q1 = b * S * P, b * S * P + Na * P, (b + 1) * S * P
                if Nq > 0:
                    self._reloc_block(pr, x, sc, rowmap_t[l, b], Na * Pp, q0, q1, Nq, P, rope, posctx, dtype, dev)
                self._global_block(pg, x, sc, a0, q0, rope, posctx)
            if l in out_maps:  # reloc half, :403-413
                om = out_maps[l]
                for b in range(B):
                    ops.copy_rows(om[b].view(Nq * P, 2 * C)[:, C:], x[b * S * P + Na * P:(b + 1) * S * P], Nq * P)
            if l == self.depth - 1:
                ops.copy_rows(cam_flat[:, C:], x, B * Na, rowmap=anchor_rows0)

        output_dict: Dict[int, torch.Tensor] = dict(out_maps)
        assert (self.depth - 1 in output_dict) or Nq == 0, \
            f"Please make sure the last layer ({self.depth - 1}) is in the output_dict: {output_dict.keys()}"
        if Nq > 0:
            output_dict[-1] = output_dict[self.depth - 1]
        return output_dict, self.patch_start_idx, cam_last

    # ------------------------------------------------------------------ stacks
    def _reloc_block(self, pb, x, sc, rowmap, n_sub, q0, q1, Nq, P, rope, posctx, dtype, dev):
        """global_reloc Block for one batch item, aggregator.py:672-741 (query rows only)."""
        C = pb.dim
        xn_sub = self._ws.get("xn_sub", n_sub, C, dtype, dev)
        kv_sub = self._ws.get("kv_sub", n_sub, 2 * C, dtype, dev)
        ops.layernorm(x, pb.ln1_w, pb.ln1_b, pb.eps, xn_sub, rowmap=rowmap, rows=n_sub)
        epi = runtime.qkv_params(pb, rope, pos_rowmap=rowmap, **posctx)
        if epi is None:
            ops.gemm(xn_sub, pb.w_qkv[C:], kv_sub, _lib.SR_EPI_BIAS, bias=pb.b_qkv[C:] if pb.b_qkv is not None else None)
        else:
            epi["col_offset"] = C
            ops.gemm(xn_sub, pb.w_qkv[C:], kv_sub, _lib.SR_EPI_QKV,
                     bias=pb.b_qkv[C:] if pb.b_qkv is not None else None, qkv=epi)

        def attend(qkv, o):
            ops.attention(qkv[:, 0:C], kv_sub[:, 0:C], kv_sub[:, C:2 * C], o, heads=pb.heads, head_dim=pb.head_dim,
                          batch=Nq, lq=P, q_bstride=P, l0=n_sub, k0_bstride=0,
                          k1=qkv[:, C:2 * C], v1=qkv[:, 2 * C:3 * C], l1=P, k1_bstride=P, tag="attn_reloc")

        runtime.run_block(pb, x, q0, q1, sc, attend, runtime.qkv_params(pb, rope, pos_row_base=q0, **posctx))

    def _global_block(self, pb, x, sc, a0, a1, rope, posctx):
        """global Block over every anchor token of one batch item, aggregator.py:743-769."""
        C = pb.dim
        L = a1 - a0

        def attend(qkv, o):
            ops.attention(qkv[:, 0:C], qkv[:, C:2 * C], qkv[:, 2 * C:3 * C], o, heads=pb.heads,
                          head_dim=pb.head_dim, batch=1, lq=L, q_bstride=0, l0=L, k0_bstride=0, tag="attn_global")

        runtime.run_block(pb, x, a0, a1, sc, attend, runtime.qkv_params(pb, rope, pos_row_base=a0, **posctx))
