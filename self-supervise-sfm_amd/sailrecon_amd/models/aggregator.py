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
import os
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
        # BASELINE C5 "fp8 QKV": the global blocks' q.k^T in block-scaled e4m3 (ops.attention_qk8);
        # opt-in (set_fp8_global or SR_FP8_GLOBAL=1), no reference output pins its precision
        self.fp8_global = os.environ.get("SR_FP8_GLOBAL", "0") in ("1", "qkv")
        self.fp8_v = os.environ.get("SR_FP8_GLOBAL", "0") == "qkv"
        self._fp8_ws = None
        # frame sharding: global attention starts on the local anchors' K/V while the remote
        # anchors' K/V are still being gathered, then merges the two passes by their LSEs
        # (SR_SHARD_OVERLAP=0: wait for the gather, one pass over every anchor)
        self.shard_overlap = os.environ.get("SR_SHARD_OVERLAP", "1") != "0"

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
        # two-phase relocalisation (attention.py:40-100, aggregator.py:435-578): anchor-subsample
        # K|V of every global_reloc layer, kept in HBM (the reference round-trips it via the CPU)
        self.kv_cache = kv_cache
        self._kv_cache_layers: Optional[List[torch.Tensor]] = None

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

    # ------------------------------------------------------------------ multi-GPU
    def set_frame_sharding(self, group=None):
        """Shard frames across the ranks of ``group`` (torch.distributed, RCCL on ROCm).

        Rank r of G owns a contiguous, balanced slice of no_reloc_list and of reloc_list
        (``shard_range``: counts differ by at most one; uneven splits are exact, no padded
        frames ever enter a softmax).  DINO, frame blocks, subsampling and every per-token GEMM
        stay local; the global block all-gathers K/V of the anchors (attending to the local
        anchors while the gather is in flight, then to the remote ones, merged by LSE), the
        global_reloc block all-gathers the anchor-subsample K/V, and the camera head runs
        replicated on gathered camera tokens.  Every rank needs >= 1 anchor;
        a rank may own no query frame.  The subsample generator is re-seeded identically on every
        rank (broadcast from rank 0) so the draws do not depend on the world size.
        ``group=None`` disables sharding."""
        self._shard_group = group
        if isinstance(group, RankSim):  # one rank's workload without peers (timing rehearsal)
            return
        if group is not None:
            seed = torch.randint(0, 2 ** 62, (1,), dtype=torch.int64)
            dist = torch.distributed
            if dist.get_backend(group) == "nccl":
                seed = seed.cuda()
            dist.broadcast(seed, src=dist.get_global_rank(group, 0) if hasattr(dist, "get_global_rank") else 0,
                           group=group)
            self.generator.manual_seed(int(seed.item()))

    def _world(self):
        g = getattr(self, "_shard_group", None)
        if g is None:
            return None, 1, 0
        if isinstance(g, RankSim):
            return g, g.world, g.rank
        return g, torch.distributed.get_world_size(g), torch.distributed.get_rank(g)

    # ------------------------------------------------------------------ forward
    def _embed(self, imgs: torch.Tensor, F_: int, H: int, W: int, ftype_t_fn, dtype) -> Tuple[torch.Tensor, object]:
        """Image normalise + DINO patch embed (+ its blocks and final norm) + aggregator special
        tokens (aggregator.py:267-299): fills the residual stream x [F_*P, C] of the workspace."""
        dev = imgs.device
        C = self.embed_dim
        ps = self.patch_size
        gh, gw = H // ps, W // ps
        n_patch = gh * gw
        psi = self.patch_start_idx
        P = n_patch + psi
        R = F_ * P
        ws = self._ws
        hidden = self.frame_blocks[0].mlp.fc1.out_features
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
                 patch=dict(seg_rows=n_patch, seg_stride=P, seg_offset=psi, row_add=row_add), tag="gemm")
        if is_dino:
            nreg_d = dino.num_register_tokens
            if 1 + nreg_d != psi:
                raise NotImplementedError("DINO register count must equal the aggregator's")
            # DINO's cls (+ its pos-embed row) and register rows, and an all-zero frame-type table:
            # parameter preprocessing, built once per resolution (no torch kernels per forward)
            key = ("dino_tokens", H, W, F_, str(dev), dino.cls_token._version, dino.register_tokens._version,
                   dino.pos_embed._version)
            if key not in self._packed:
                dtab = torch.cat([(dino.cls_token[0, 0] + pos_tab[0])[None], dino.register_tokens[0]], 0)
                self._packed = {k: v for k, v in self._packed.items() if not (isinstance(k, tuple) and
                                                                             k[0] == "dino_tokens")}
                self._packed[key] = (dtab.detach().float().contiguous()[None],
                                     torch.zeros(F_, 1, dtype=torch.int32, device=dev))
            dtab, zero_t = self._packed[key]
            ops.set_special_tokens(x, F_, P, dtab, zero_t)
            pending = []  # fc2 residual of block i folded into block i+1's LN1 (runtime.Pending)
            nblk = len(dino.blocks)
            for i, blk in enumerate(dino.blocks):
                pb = blk.packed(dtype)
                qs = runtime.q_prescale(pb)  # c*q rounded once by the QKV GEMM (runtime.q_prescale)
                p = runtime.run_block(pb, x, 0, R, sc, runtime.frame_attend(pb, F_, P, tail_readable=True,
                                                                            q_scaled=qs > 0),
                                      runtime.qkv_params(pb, None, prescale=True), pending=pending,
                                      defer=i < nblk - 1, q_scale=qs)
                if p is not None:
                    pending.append(p)
            assert not pending
            ops.layernorm(x, dino.norm.weight, dino.norm.bias, dino.norm.eps, x)  # in place (row-local)

        # ---- aggregator special tokens, aggregator.py:287-299 (type by ORIGINAL frame index)
        ops.set_special_tokens(x, F_, P, misc["special"], ftype_t_fn())
        return x, sc


    def forward(self, images: torch.Tensor, no_reloc_list: list, reloc_list: list,
                fix_rank: Union[int, None] = None) -> Tuple[Dict[int, torch.Tensor], int, torch.Tensor]:
        B, S, C_in, H, W = images.shape
        num_recon, num_reloc = len(no_reloc_list), len(reloc_list)
        self.num_recon = num_recon
        if C_in != 3:
            raise ValueError(f"Expected 3 input channels, got {C_in}")
        runtime.require_device(images, "Aggregator")
        if sorted(list(no_reloc_list) + list(reloc_list)) != list(range(S)):
            raise ValueError("no_reloc_list and reloc_list must be disjoint and cover every frame "
                             f"(S={S}, got {list(no_reloc_list)} / {list(reloc_list)}); the reference's "
                             "block mask (aggregator.py:302-311) assumes the same")
        if num_recon == 0:
            raise ValueError("at least one anchor (no_reloc) frame is required")
        ps = self.patch_size
        assert H % ps == 0 and W % ps == 0, f"image size {H}x{W} is not a multiple of the patch size {ps}"
        group, G, r = self._world()
        Na, Nq = num_recon, num_reloc
        if self.kv_cache and Nq > 0:
            raise NotImplementedError("a kv_cache aggregator runs anchors only here (SailRecon.tmp_forward) and "
                                      "queries through forward_with_cache (SailRecon.reloc), like the reference")
        fill_cache = self.kv_cache  # anchors-only pass: keep every layer's anchor-subsample K|V
        if G > 1 and (B != 1 or Na < G):
            raise ValueError(f"frame sharding over {G} ranks needs B == 1 and at least one anchor frame per "
                             f"rank (got B={B}, Na={Na})")
        a_start, Na_l = shard_range(Na, G, r)
        q_start, Nq_l = shard_range(Nq, G, r)
        a_counts = [shard_range(Na, G, j)[1] for j in range(G)]
        q_counts = [shard_range(Nq, G, j)[1] for j in range(G)]
        my_anchors = list(no_reloc_list)[a_start:a_start + Na_l]
        my_queries = list(reloc_list)[q_start:q_start + Nq_l]
        S_l = Na_l + Nq_l

        dev = images.device
        dtype = runtime.compute_dtype(self.compute_dtype)
        C, nh = self.embed_dim, self.num_heads
        gh, gw = H // ps, W // ps
        n_patch = gh * gw
        psi = self.patch_start_idx
        P = n_patch + psi
        F_ = B * S_l
        R = F_ * P
        ws = self._ws
        hidden = self.frame_blocks[0].mlp.fc1.out_features

        # ---- internal (local) frame order: anchors then queries, per batch item
        order = my_anchors + my_queries
        imgs = images if order == list(range(S)) else images[:, order]
        imgs = imgs.reshape(F_, 3, H, W).float().contiguous()

        need_sub = Nq > 0 or fill_cache
        if fill_cache and B != 1:
            raise NotImplementedError("kv_cache needs B == 1 (aggregator.py:452)")
        host = {}

        def host_tables():
            """Every per-forward host table in ONE pinned H2D copy, built once _embed has queued its GPU
            work (so the subsample draws overlap DINO): the frame types (aggregator.py:287-299, by
            ORIGINAL frame index), the anchors' camera-token rows and the per-layer subsample row maps
            (aggregator.py:277-285, 580-626).  Returns the frame-type view."""
            if fix_rank is not None:
                self.rank = min(fix_rank, n_patch)
            else:
                lo, hi = min(self.min_rank, n_patch // 2), max(self.min_rank, n_patch // 2)
                self.rank = int(torch.randint(lo, hi, (1,), generator=self.generator).item())
            Pp = min(self.rank + psi, P)
            # the reference draws at every layer even without queries (select_scene_repe_for_reloc,
            # aggregator.py:351-357), so the generator advances identically
            idx = self.draw_subsample(self.depth, B, Na, n_patch, self.rank)  # every rank draws all anchors
            self.last_subsample_indices = torch.from_numpy(idx)
            ftype = np.array(sum(([0 if a == 0 else 1 for a in my_anchors] + [2] * Nq_l for _ in range(B)), []),
                             dtype=np.int32)
            anchors = np.array([b * S_l * P + a * P for b in range(B) for a in range(Na_l)], dtype=np.int32)
            parts = [ftype, anchors]
            if need_sub:
                idx = idx[:, :, a_start:a_start + Na_l]                       # this rank's anchors
                base = (np.arange(B) * S_l * P)[None, :, None, None] + (np.arange(Na_l) * P)[None, None, :, None]
                sel = base + psi + idx                                        # [depth, B, Na_l, rank]
                spec = np.broadcast_to(base + np.arange(psi)[None, None, None, :], (self.depth, B, Na_l, psi))
                parts.append(np.concatenate([spec, sel], axis=-1).astype(np.int32).reshape(-1))
            buf = runtime.to_device(torch.from_numpy(np.concatenate(parts)), dev)
            n0, n1 = len(ftype), len(ftype) + len(anchors)
            host.update(Pp=Pp, anchor_rows0=buf[n0:n1],
                        rowmap_t=buf[n1:].view(self.depth, B, Na_l * Pp) if need_sub else None)
            return buf[:n0]

        x, sc = self._embed(imgs, F_, H, W, ftype_t_fn=host_tables, dtype=dtype)
        Pp, rowmap_t, anchor_rows0 = host["Pp"], host["rowmap_t"], host["anchor_rows0"]
        if fill_cache:
            self._kv_cache_layers = [None] * self.depth
        rope = self.rope.tables(C // nh, max(gh, gw) + 1, dev) if self.rope is not None else None
        posctx = dict(tokens_per_frame=P, patch_start=psi, grid_w=gw)

        # ---- outputs (this rank's query frames)
        out_maps: Dict[int, torch.Tensor] = {}
        if Nq > 0:
            for l in self.intermediate_layer_idx:
                out_maps[l] = torch.empty(B, Nq_l, P, 2 * C, device=dev, dtype=torch.float32)
        cam_loc = torch.empty(B, Na_l, 2 * C, device=dev, dtype=torch.float32)
        cam_flat = cam_loc.view(B * Na_l, 2 * C)

        # ---- alternating layers, aggregator.py:339-423
        pending = []  # the global / reloc blocks' fc2 residuals, folded into the next frame block's LN1
        for l in range(self.depth):
            pb = self.frame_blocks[l].packed(dtype)
            runtime.run_block(pb, x, 0, R, sc, runtime.frame_attend(pb, F_, P, tail_readable=True, q_scaled=_qs(pb)),
                              runtime.qkv_params(pb, rope, prescale=True, pos_row_base=0, **posctx), pending=pending,
                              q_scale=runtime.q_prescale(pb))
            if l in out_maps and Nq_l > 0:  # frame half of the intermediate, :403-413
                for b in range(B):
                    ops.copy_rows(out_maps[l][b].view(Nq_l * P, 2 * C)[:, :C],
                                  x[b * S_l * P + Na_l * P:(b + 1) * S_l * P], Nq_l * P)
            if l == self.depth - 1:  # :414-423 frame half
                ops.copy_rows(cam_flat[:, :C], x, B * Na_l, rowmap=anchor_rows0)
            pr = self.global_reloc_blocks[l].packed(dtype)
            pg = self.global_blocks[l].packed(dtype)
            # the next reader of x after this layer's global / reloc blocks is the next frame block's LN1,
            # unless an output map or the camera tokens copy x first
            defer = l + 1 < self.depth and l not in out_maps and not fill_cache and \
                os.environ.get("SR_CONCURRENT_STACKS", "0") != "1"
            for b in range(B):
                a0, q0, q1 = b * S_l * P, b * S_l * P + Na_l * P, (b + 1) * S_l * P
                pending += self._layer_global(pr, pg, x, sc, rowmap_t[l, b] if need_sub else None, Pp, a0, q0, q1,
                                              Nq_l, P, rope, posctx, dtype, dev, group, G, r, a_counts, need_sub,
                                              cache_layer=l if fill_cache else None, defer=defer)
            if l in out_maps and Nq_l > 0:  # reloc half
                for b in range(B):
                    ops.copy_rows(out_maps[l][b].view(Nq_l * P, 2 * C)[:, C:],
                                  x[b * S_l * P + Na_l * P:(b + 1) * S_l * P], Nq_l * P)
            if l == self.depth - 1:
                ops.copy_rows(cam_flat[:, C:], x, B * Na_l, rowmap=anchor_rows0)

        output_dict: Dict[int, torch.Tensor] = dict(out_maps)
        assert (self.depth - 1 in output_dict) or Nq == 0, \
            f"Please make sure the last layer ({self.depth - 1}) is in the output_dict: {output_dict.keys()}"
        if Nq > 0:
            output_dict[-1] = output_dict[self.depth - 1]
        if G > 1:
            # camera head inputs for every frame: anchor camera tokens and query camera tokens
            cam_last = torch.empty(B * Na, 2 * C, device=dev, dtype=torch.float32)
            works = gather_rows(cam_last, cam_loc.view(B * Na_l, 2 * C), a_counts, group, r)
            if Nq > 0:
                qcam = torch.empty(B * Nq, 2 * C, device=dev, dtype=torch.float32)
                works += gather_rows(qcam, output_dict[-1][:, :, 0].reshape(B * Nq_l, 2 * C).contiguous(), q_counts,
                                     group, r)
                self.last_query_cam_tokens = qcam.view(B, Nq, 2 * C)
            for w in works:
                w.wait()
            cam_last = cam_last.view(B, Na, 2 * C)
        else:
            cam_last = cam_loc
            self.last_query_cam_tokens = output_dict[-1][:, :, 0] if Nq > 0 else None
        return output_dict, self.patch_start_idx, cam_last

    # ------------------------------------------------------------------ two-phase relocalisation
    def clear_kv_cache(self) -> None:
        """attention.py:48-60 for every global_reloc block."""
        self._kv_cache_layers = None

    def forward_with_cache(self, images: torch.Tensor, cameras: torch.Tensor = None, camera_dropout: float = False,
                           fix_rank: Union[int, None] = None) -> Tuple[Dict[int, torch.Tensor], int]:
        """aggregator.py:435-578: relocalise query frames against the anchors cached by an
        anchors-only ``forward`` of a ``kv_cache=True`` aggregator.  Every frame of ``images``
        is a query: reloc special tokens, frame blocks, and per layer the global_reloc block
        over [cached anchor-subsample K|V ; the frame's own tokens] (the reference's cache
        concatenation + block mask, attention.py:80-100, aggregator.py:497-509).  Returns
        (output_dict {inter layers, -1: [1, S, P, 2C]}, patch_start_idx)."""
        B, S, C_in, H, W = images.shape
        assert B == 1, "Batch size must be 1 for this model"
        if C_in != 3:
            raise ValueError(f"Expected 3 input channels, got {C_in}")
        runtime.require_device(images, "Aggregator.forward_with_cache")
        if self._kv_cache_layers is None or any(t is None for t in self._kv_cache_layers):
            raise RuntimeError("forward_with_cache needs a filled cache: run the anchors-only forward first "
                               "(SailRecon.tmp_forward)")
        if self._world()[1] > 1:
            raise NotImplementedError("forward_with_cache under frame sharding")
        ps = self.patch_size
        assert H % ps == 0 and W % ps == 0, f"image size {H}x{W} is not a multiple of the patch size {ps}"
        if fix_rank is not None:
            self.rank = fix_rank
        dev = images.device
        dtype = runtime.compute_dtype(self.compute_dtype)
        if self._kv_cache_layers[0].dtype != dtype:
            raise RuntimeError(f"the cache was built in {self._kv_cache_layers[0].dtype}, this pass computes in "
                               f"{dtype}: run both phases under the same autocast setting")
        C, nh = self.embed_dim, self.num_heads
        gh, gw = H // ps, W // ps
        psi = self.patch_start_idx
        P = gh * gw + psi
        F_ = S
        R = F_ * P
        n_sub = self._kv_cache_layers[0].shape[0]
        imgs = images.reshape(F_, 3, H, W).float().contiguous()
        x, sc = self._embed(imgs, F_, H, W, ftype_t_fn=lambda: torch.full((F_,), 2, device=dev, dtype=torch.int32),
                            dtype=dtype)
        rope = self.rope.tables(C // nh, max(gh, gw) + 1, dev) if self.rope is not None else None
        posctx = dict(tokens_per_frame=P, patch_start=psi, grid_w=gw)
        out_maps = {l: torch.empty(1, S, P, 2 * C, device=dev, dtype=torch.float32) for l in self.intermediate_layer_idx}
        for l in range(self.depth):
            pb = self.frame_blocks[l].packed(dtype)
            runtime.run_block(pb, x, 0, R, sc, runtime.frame_attend(pb, F_, P, tail_readable=True, q_scaled=_qs(pb)),
                              runtime.qkv_params(pb, rope, prescale=True, pos_row_base=0, **posctx),
                              q_scale=runtime.q_prescale(pb))
            if l in out_maps:
                ops.copy_rows(out_maps[l][0].view(R, 2 * C)[:, :C], x, R)
            pr = self.global_reloc_blocks[l].packed(dtype)
            kv = self._kv_cache_layers[l]

            def attend_cached(qkv, o, kv=kv, pr=pr):
                ops.attention(qkv[:, 0:C], kv[:, 0:C], kv[:, C:2 * C], o, heads=pr.heads, head_dim=pr.head_dim,
                              batch=F_, lq=P, q_bstride=P, l0=n_sub, k0_bstride=0, k1=qkv[:, C:2 * C],
                              v1=qkv[:, 2 * C:3 * C], l1=P, k1_bstride=P, tag="attn_reloc",
                              key_norm_max=runtime.key_norm_bound(pr),
                              query_norm_max=runtime.query_norm_bound(pr), q_scaled=_qs(pr))
            runtime.run_block(pr, x, 0, R, sc, attend_cached,
                              runtime.qkv_params(pr, rope, prescale=True, pos_row_base=0, **posctx),
                              q_scale=runtime.q_prescale(pr))
            if l in out_maps:
                ops.copy_rows(out_maps[l][0].view(R, 2 * C)[:, C:], x, R)
        assert self.depth - 1 in out_maps, \
            f"Please make sure the last layer ({self.depth - 1}) is in the output_dict: {out_maps.keys()}"
        output_dict: Dict[int, torch.Tensor] = dict(out_maps)
        output_dict[-1] = output_dict[self.depth - 1]
        return output_dict, self.patch_start_idx

    # ------------------------------------------------------------------ stacks
    def _layer_global(self, pr, pg, x, sc, rowmap, Pp, a0, q0, q1, Nq_l, P, rope, posctx, dtype, dev,
                      group, G, r, a_counts, need_sub, cache_layer=None, defer=False) -> list:
        """global_reloc (queries, aggregator.py:672-741) + global (anchors, :743-769) blocks of
        one layer for one batch item.  With G > 1 the anchor K/V and the anchor-subsample K/V
        are gathered asynchronously (``gather_rows``; ``a_counts`` = anchor frames per rank):
        the subsample K/V behind the query-side QKV GEMM, the anchor K/V behind the whole reloc
        block and the local-anchor attention pass.  ``defer``: the two blocks' fc2 residuals are
        returned as runtime.Pending updates for the next frame block's LN1 (else [])."""
        out = []

        def keep(p):
            if p is not None:
                out.append(p)
        C = pg.dim
        ws = self._ws
        La_l = q0 - a0                 # local anchor tokens
        La = sum(a_counts) * P         # all anchor tokens
        n_sub = (q0 - a0) // P * Pp    # local anchor-subsample rows
        n_sub_all = sum(a_counts) * Pp
        work_sub, work_kv = [], []
        paired = G == 1 and self._paired_attention(pr, pg, dtype, Nq_l * P, q0 - a0, n_sub_all)
        # paired: the subsample K/V projection joins the queries' and anchors' QKV GEMMs in one
        # grouped launch below (its LayerNorm still reads x here, before the global block updates it)
        defer_kv = paired and cache_layer is None and need_sub
        if need_sub:
            # anchor-subsample K/V (reads x before the global block updates the anchors)
            xn_sub = ws.get("xn_sub", n_sub, C, dtype, dev)
            if G > 1:  # separate send buffer: no aliasing between collective input and output
                kv_sub = ws.get("kv_sub_loc", n_sub, 2 * C, dtype, dev)
                kv_sub_all = ws.get("kv_sub", n_sub_all, 2 * C, dtype, dev)
            else:
                kv_sub = kv_sub_all = ws.get("kv_sub", n_sub, 2 * C, dtype, dev)
            ops.layernorm(x, pr.ln1_w, pr.ln1_b, pr.eps, xn_sub, rowmap=rowmap, rows=n_sub)
            if not defer_kv:
                self._kv_gemm(pr, xn_sub, kv_sub, rope, dict(pos_rowmap=rowmap, **posctx))
            if G > 1:
                work_sub = gather_rows(kv_sub_all, kv_sub, [c * Pp for c in a_counts], group, r)
            if cache_layer is not None:  # two-phase reloc: every anchor's subsample K|V of this layer
                _wait(work_sub)
                self._kv_cache_layers[cache_layer] = kv_sub_all.clone()
        if G > 1:
            # global block, first half: LN1 + Q GEMM locally, K/V straight into this rank's slot
            xs = x[a0:q0]
            xn, qkv = sc.xn[a0:q0], sc.qkv[a0:q0]
            kv_all = ws.get("kv_all", La, 2 * C, dtype, dev)
            kv_loc = ws.get("kv_loc", La_l, 2 * C, dtype, dev)
            ops.layernorm(xs, pg.ln1_w, pg.ln1_b, pg.eps, xn)
            epi = runtime.qkv_params(pg, rope, prescale=True, pos_row_base=a0, **posctx)
            epi_kv = runtime.qkv_params(pg, rope, pos_row_base=a0, **posctx)
            probs = []
            if epi is not None and epi_kv is not None:
                epi_kv["col_offset"] = C
                probs = [dict(a=xn, w=pg.w_qkv[:C], out=qkv[:, :C], bias=_sl(pg.b_qkv, 0, C), qkv=epi),
                         dict(a=xn, w=pg.w_qkv[C:], out=kv_loc, bias=_sl(pg.b_qkv, C, 3 * C), qkv=epi_kv)]
            if probs and ops.gemm_group_eligible(probs):
                # Q and K/V as ONE grouped launch: at G = 8 a rank's 5,496 anchor rows are 88 + 176
                # tiles of 256^2, each under one workgroup round on its own
                ops.gemm_group(probs, _lib.SR_EPI_QKV, tag="gemm")
            else:
                runtime.qkv_gemm(pg, xn, pg.w_qkv[:C], qkv[:, :C], _sl(pg.b_qkv, 0, C), epi, runtime.q_prescale(pg))
                self._kv_gemm(pg, xn, kv_loc, rope, dict(pos_row_base=a0, **posctx))
            work_kv = gather_rows(kv_all, kv_loc, [c * P for c in a_counts], group, r)
        if paired:
            # G == 1, bf16: the queries' and anchors' QKV projections (and the anchor-subsample K/V
            # one) as ONE grouped GEMM launch, then the global block's attention (anchors against
            # themselves) and the split reloc block's subsample pass (queries against the anchor
            # subsample) in ONE launch of the hand-scheduled sweep (sr_attention_pair): each time the
            # second problem fills the CUs the first one's last workgroup round leaves idle; then the
            # reloc own-frame pass folds the subsample pass in, and both blocks' tails follow
            rows, La = Nq_l * P, q0 - a0
            n_full = n_sub_all // 64 * 64
            epi_r = runtime.qkv_params(pr, rope, prescale=True, pos_row_base=q0, **posctx)
            epi_g = runtime.qkv_params(pg, rope, prescale=True, pos_row_base=a0, **posctx)
            epi_s = runtime.qkv_params(pr, rope, pos_rowmap=rowmap, **posctx) if defer_kv else None
            if epi_s is not None:
                epi_s["col_offset"] = C
            probs = [dict(a=sc.xn[q0:q1], w=pr.w_qkv, out=sc.qkv[q0:q1], bias=pr.b_qkv, qkv=epi_r),
                     dict(a=sc.xn[a0:q0], w=pg.w_qkv, out=sc.qkv[a0:q0], bias=pg.b_qkv, qkv=epi_g)]
            if defer_kv:
                probs.append(dict(a=xn_sub, w=pr.w_qkv[C:], out=kv_sub_all, bias=_sl(pr.b_qkv, C, 3 * C), qkv=epi_s))
            if all(p_["qkv"] is not None for p_ in probs) and ops.gemm_group_eligible(probs):
                ops.layernorm(x[q0:q1], pr.ln1_w, pr.ln1_b, pr.eps, sc.xn[q0:q1])
                ops.layernorm(x[a0:q0], pg.ln1_w, pg.ln1_b, pg.eps, sc.xn[a0:q0])
                ops.gemm_group(probs, _lib.SR_EPI_QKV, tag="gemm")
            else:
                runtime.run_block_head(pr, x, q0, q1, sc, epi_r, runtime.q_prescale(pr))
                runtime.run_block_head(pg, x, a0, q0, sc, epi_g, runtime.q_prescale(pg))
                if defer_kv:
                    self._kv_gemm(pr, xn_sub, kv_sub_all, rope, dict(pos_rowmap=rowmap, **posctx))
            qkv_r, qkv_g = sc.qkv[q0:q1], sc.qkv[a0:q0]
            o_a, lse_a = ops.key_split_workspace(dev, 1, rows, C, pr.heads, name="reloc_split")
            lse_a = lse_a[0]
            pa = dict(q=qkv_g[:, 0:C], k0=qkv_g[:, C:2 * C], v0=qkv_g[:, 2 * C:3 * C], o=sc.o[a0:q0], lq=La, l0=La,
                      key_norm_max=runtime.key_norm_bound(pg), query_norm_max=runtime.query_norm_bound(pg),
                      q_scaled=_qs(pg))
            pb = dict(q=qkv_r[:, 0:C], k0=kv_sub_all[:n_full, 0:C], v0=kv_sub_all[:n_full, C:2 * C], o=o_a, lq=rows,
                      l0=n_full, key_norm_max=runtime.key_norm_bound(pr), query_norm_max=runtime.query_norm_bound(pr),
                      lse=lse_a.view(-1), q_scaled=_qs(pr))
            if ops.PAIR_VT:
                # both problems' V as pre-transposed tiles: one ds_read_b128 per P.V fragment in the sweep
                for p_, name, blk in ((pa, "vt_g", pg), (pb, "vt_s", pr)):
                    p_["vt"] = ops.vt_tiles(p_["v0"], p_["l0"], blk.heads,
                                            ws.get(name, *ops.vt_tile_shape(p_["l0"], blk.heads), dtype, dev),
                                            tag="vt_tiles")
            ops.attention_pair(pa, pb, heads=pg.heads, head_dim=pg.head_dim, tag="attn_global")
            self._reloc_own_pass(pr, qkv_r, kv_sub_all, sc.o[q0:q1], o_a, lse_a, Nq_l, P, n_sub_all, n_full)
            if runtime.group_tails_wanted(max(q1 - q0, q0 - a0)):
                out.extend(runtime.run_block_tails([(pr, q0, q1), (pg, a0, q0)], x, sc, defer=defer))
            else:
                keep(runtime.run_block_tail(pr, x, q0, q1, sc, defer=defer))
                keep(runtime.run_block_tail(pg, x, a0, q0, sc, defer=defer))
            return out
        # G == 1: the reloc block (query rows) and the global block (anchor rows) are independent.
        # SR_CONCURRENT_STACKS=1 runs the reloc block on a side stream so that each could fill the
        # other's last partial wave.  Round 1: 3% SLOWER at N=32 (68.7 -> 66.7 views/s).  Round 3,
        # with the one-workgroup-per-CU asm attention and the split reloc: 0.8 % faster (409.4 / 409.1
        # vs 411.9 / 413.2 ms, one box, interleaved; C2 / C3 goldens pass), but the kernels of the two
        # streams then overlap, so no per-kernel time (HIP events or rocprofv3) measures a kernel any
        # more -- the roofline of the dominant kernel reads 0.40 instead of 0.50.  Off by default,
        # so that the bench's roofline stays a measurement of the kernel.
        side = self._side_stream(dev) if (G == 1 and Nq_l > 0 and a0 < q0) else None
        # frame-sharded: the reloc block's tail waits for the global attention and runs grouped with
        # the global block's (runtime.run_block_tails: one launch per GEMM stage over both row ranges)
        group_tails = G > 1 and Nq_l > 0 and runtime.group_tails_wanted(max(q1 - q0, q0 - a0))
        # ... and with SR_SHARD_CONCURRENT=1 its attention runs on a second stream beside the global
        # attention's key-split passes: at G = 8 both under-fill the chip on their own
        shard_side = (self._stream2(dev) if group_tails and _SHARD_CONCURRENT and torch.device(dev).type == "cuda"
                      else None)
        if Nq_l > 0:
            def attend_reloc(qkv, o):
                _wait(work_sub)
                rows = Nq_l * P
                kb, qb = runtime.key_norm_bound(pr), runtime.query_norm_bound(pr)
                if self._split_reloc(dtype, rows, n_sub_all):
                    # two passes merged by their LSEs (the union of the two key sets, exactly): every
                    # query row against the shared anchor subsample's whole 64-key tiles as ONE long
                    # query set (the hand-scheduled sweep, sr_attn.hip), then each query frame against
                    # the subsample's last partial tile (shared segment 0) and itself (segment 1) on
                    # the compiled sweep, whose epilogue folds the first pass in (sr_attn_desc.merge_o)
                    n_full = n_sub_all // 64 * 64
                    o_a, lse_a = ops.key_split_workspace(dev, 1, rows, C, pr.heads, name="reloc_split")
                    lse_a = lse_a[0]
                    ops.attention(qkv[:, 0:C], kv_sub_all[:n_full, 0:C], kv_sub_all[:n_full, C:2 * C],
                                  o_a, heads=pr.heads, head_dim=pr.head_dim, batch=1, lq=rows,
                                  q_bstride=0, l0=n_full, k0_bstride=0, tag="attn_reloc", key_norm_max=kb,
                                  query_norm_max=qb,
                                  lse=lse_a.view(-1), tail_readable=True, q_scaled=_qs(pr))
                    self._reloc_own_pass(pr, qkv, kv_sub_all, o, o_a, lse_a, Nq_l, P, n_sub_all, n_full)
                    return
                ops.attention(qkv[:, 0:C], kv_sub_all[:, 0:C], kv_sub_all[:, C:2 * C], o, heads=pr.heads,
                              head_dim=pr.head_dim, batch=Nq_l, lq=P, q_bstride=P, l0=n_sub_all, k0_bstride=0,
                              k1=qkv[:, C:2 * C], v1=qkv[:, 2 * C:3 * C], l1=P, k1_bstride=P, tag="attn_reloc",
                              key_norm_max=kb, query_norm_max=qb, tail_readable=True, q_scaled=_qs(pr))
            if side is not None:
                side.wait_stream(torch.cuda.current_stream(dev))  # frame block + subsample K/V are done
                with torch.cuda.stream(side):
                    runtime.run_block(pr, x, q0, q1, sc, attend_reloc,
                                      runtime.qkv_params(pr, rope, prescale=True, pos_row_base=q0, **posctx),
                                      q_scale=runtime.q_prescale(pr))
            elif group_tails:  # the tail joins the global block's in run_block_tails below
                runtime.run_block_head(pr, x, q0, q1, sc,
                                       runtime.qkv_params(pr, rope, prescale=True, pos_row_base=q0, **posctx),
                                       runtime.q_prescale(pr))
                if shard_side is not None:
                    shard_side.wait_stream(torch.cuda.current_stream(dev))  # the reloc QKV is done
                    with torch.cuda.stream(shard_side):  # (its wait on the subsample gather too)
                        attend_reloc(sc.qkv[q0:q1], sc.o[q0:q1])
                else:
                    attend_reloc(sc.qkv[q0:q1], sc.o[q0:q1])
            else:
                keep(runtime.run_block(pr, x, q0, q1, sc, attend_reloc,
                                       runtime.qkv_params(pr, rope, prescale=True, pos_row_base=q0, **posctx),
                                       defer=defer, q_scale=runtime.q_prescale(pr)))
        _wait(work_sub)  # a rank without query frames still fed the others (send buffer reuse)
        if G > 1:
            o, q = sc.o[a0:q0], sc.qkv[a0:q0, 0:C]
            fp8 = self.fp8_global and pg.head_dim == 64 and q.dtype == torch.bfloat16
            if self.shard_overlap and not fp8:
                self._global_attention_sharded(q, kv_loc, kv_all, o, pg, La_l, La, sum(a_counts[:r]) * P, work_kv)
            else:
                _wait(work_kv)
                self._global_attention(q, kv_all[:, 0:C], kv_all[:, C:2 * C], o, pg, La_l, La)
            if shard_side is not None:
                torch.cuda.current_stream(dev).wait_stream(shard_side)  # join before the grouped tails
            if group_tails:
                out.extend(runtime.run_block_tails([(pr, q0, q1), (pg, a0, q0)], x, sc, defer=defer))
            else:
                keep(runtime.run_block_tail(pg, x, a0, q0, sc, defer=defer))
        else:
            def attend_global(qkv, o):
                self._global_attention(qkv[:, 0:C], qkv[:, C:2 * C], qkv[:, 2 * C:3 * C], o, pg, La, La)
            keep(runtime.run_block(pg, x, a0, q0, sc, attend_global,
                                   runtime.qkv_params(pg, rope, prescale=True, pos_row_base=a0, **posctx),
                                   defer=defer, q_scale=runtime.q_prescale(pg)))
        if side is not None:
            torch.cuda.current_stream(dev).wait_stream(side)  # join before the next frame block
        return out

    def set_fp8_global(self, enabled: bool = True, fp8_v: bool = False):
        """Global blocks' q.k^T in block-scaled fp8 (BASELINE C5); with ``fp8_v`` also V and P.V.
        Everything else stays bf16."""
        self.fp8_global = bool(enabled)
        self.fp8_v = bool(enabled and fp8_v)
        return self

    def _global_attention_sharded(self, q, kv_loc, kv_all, o, pg, lq, lk, off, work_kv):
        """softmax over every anchor's keys in two passes: the local anchors (kv_loc, ready now)
        while the gather of the others is in flight, then the remote anchors (kv_all rows outside
        [off, off + lq): up to two key segments), merged exactly by the passes' LSEs."""
        C, H, D = pg.dim, pg.heads, pg.head_dim
        kb, qb = runtime.key_norm_bound(pg), runtime.query_norm_bound(pg)
        segs = [(a, n) for a, n in ((0, off), (off + lq, lk - off - lq)) if n > 0]
        if q.dtype == torch.bfloat16:
            # every pass key-split as one slice of a stacked partials buffer (the per-rank query
            # slice alone leaves CUs idle at G >= 4), one N-way LSE merge at the end
            split = lambda n: ops.key_split_parts(dtype=q.dtype, batch=1, lq=lq, heads=H, l0=n, l1=0,  # noqa: E731
                                                  mask_mode=0)
            plan = [[kv_loc, split(lq)]] + [[kv_all[a:a + n], split(n)] for a, n in segs]
            # one sr_attn_merge_n takes at most SR_ATTN_MERGE_MAX_PARTS partials: a middle rank's two
            # remote segments can each want 8 (C3 at G = 8, ranks 3 and 4: 2 + 8 + 8), so the pass
            # with the most parts gives up half of them (its chunks double) until the total fits
            while sum(p for _, p in plan) > _lib.SR_ATTN_MERGE_MAX_PARTS:
                big = max(plan, key=lambda e: e[1])
                big[1] = max(1, big[1] // 2)
            plan = [(kv, [(0, kv.shape[0], p)]) for kv, p in plan]  # one launch of p equal chunks per pass
            total = sum(pp for _, pieces in plan for _, _, pp in pieces)
            o_parts, lse_parts = ops.key_split_workspace(q.device, total, lq, C, H, name="attn_shard")
            p0 = 0
            for i, (kv, pieces) in enumerate(plan):
                if i == 1:
                    _wait(work_kv)  # the remote anchors' K/V
                for a, m, pp in pieces:
                    ops.attention_partials(q, kv[a:a + m, 0:C], kv[a:a + m, C:2 * C],
                                           o_parts[p0 * lq:(p0 + pp) * lq], lse_parts[p0:p0 + pp], heads=H,
                                           head_dim=D, lq=lq, l0=m, parts=pp, tag="attn_global", key_norm_max=kb,
                                           query_norm_max=qb, tail_readable=_SHARD_TAIL, q_scaled=_qs(pg))
                    p0 += pp
            ops.attn_merge_n(o_parts, lse_parts, o, parts=total, rows=lq, heads=H, head_dim=D)
            return
        ws = self._ws
        lse_loc = ws.get("lse_loc", H, lq, torch.float32, q.device)
        lse_rem = ws.get("lse_rem", H, lq, torch.float32, q.device)
        o_rem = ws.get("o_rem", lq, C, o.dtype, q.device)
        ops.attention(q, kv_loc[:, 0:C], kv_loc[:, C:2 * C], o, heads=H, head_dim=D, batch=1, lq=lq, q_bstride=0,
                      l0=lq, k0_bstride=0, tag="attn_global", lse=lse_loc, key_norm_max=kb, query_norm_max=qb,
                      q_scaled=_qs(pg))
        _wait(work_kv)
        (s0, n0), (s1, n1) = segs[0], (segs[1] if len(segs) > 1 else (0, 0))
        ops.attention(q, kv_all[s0:s0 + n0, 0:C], kv_all[s0:s0 + n0, C:2 * C], o_rem, heads=H, head_dim=D, batch=1,
                      lq=lq, q_bstride=0, l0=n0, k0_bstride=0, k1=kv_all[s1:s1 + n1, 0:C] if n1 else None,
                      v1=kv_all[s1:s1 + n1, C:2 * C] if n1 else None, l1=n1, k1_bstride=0, tag="attn_global",
                      lse=lse_rem, key_norm_max=kb, query_norm_max=qb, q_scaled=_qs(pg))
        ops.attn_merge(o, lse_loc, o_rem, lse_rem, o, heads=H, head_dim=D, tag="attn_merge")

    def _global_attention(self, q, k, v, o, pg, lq, lk):
        if self.fp8_global and pg.head_dim == 64 and q.dtype == torch.bfloat16:
            if self._fp8_ws is None:
                self._fp8_ws = ops.Fp8Workspace()
            ops.attention_qk8(q, k, v, o, heads=pg.heads, batch=1, lq=lq, q_bstride=0, l0=lk, k0_bstride=0,
                              tag="attn_global", ws=self._fp8_ws, fp8_v=self.fp8_v,
                              key_norm_max=runtime.key_norm_bound(pg), q_scaled=_qs(pg))
        else:
            ops.attention(q, k, v, o, heads=pg.heads, head_dim=pg.head_dim, batch=1, lq=lq, q_bstride=0, l0=lk,
                          k0_bstride=0, tag="attn_global", key_norm_max=runtime.key_norm_bound(pg),
                          query_norm_max=runtime.query_norm_bound(pg), q_scaled=_qs(pg))

    @staticmethod
    def _reloc_own_pass(pr, qkv, kv_sub_all, o, o_a, lse_a, nq: int, P: int, n_sub_all: int, n_full: int) -> None:
        """Second pass of the split reloc attention: each query frame against the subsample's last
        partial tile (shared segment 0) and itself (segment 1), folding the subsample pass's
        (o_a, lse_a) in at its epilogue (sr_attn_desc.merge_o) -> o."""
        C, kb, qb = pr.dim, runtime.key_norm_bound(pr), runtime.query_norm_bound(pr)
        if n_full < n_sub_all:
            ops.attention(qkv[:, 0:C], kv_sub_all[n_full:, 0:C], kv_sub_all[n_full:, C:2 * C], o, heads=pr.heads,
                          head_dim=pr.head_dim, batch=nq, lq=P, q_bstride=P, l0=n_sub_all - n_full, k0_bstride=0,
                          k1=qkv[:, C:2 * C], v1=qkv[:, 2 * C:3 * C], l1=P, k1_bstride=P, tag="attn_reloc",
                          key_norm_max=kb, query_norm_max=qb, tail_readable=True, merge_o=o_a, merge_lse=lse_a,
                          q_scaled=_qs(pr))
        else:
            ops.attention(qkv[:, 0:C], qkv[:, C:2 * C], qkv[:, 2 * C:3 * C], o, heads=pr.heads, head_dim=pr.head_dim,
                          batch=nq, lq=P, q_bstride=P, l0=P, k0_bstride=P, tag="attn_reloc", key_norm_max=kb,
                          query_norm_max=qb,
                          tail_readable=True, merge_o=o_a, merge_lse=lse_a, q_scaled=_qs(pr))

    def _paired_attention(self, pr, pg, dtype, rows: int, La: int, n_sub: int) -> bool:
        """Single GPU, bf16, split reloc, a global query set that fills the chip without key
        splitting: the global attention and the reloc subsample pass in one launch
        (ops.attention_pair; SR_ATTN_PAIR=0 launches them apart)."""
        if not self._split_reloc(dtype, rows, n_sub) or self.fp8_global or La <= 0 or pg.heads != pr.heads:
            return False
        if os.environ.get("SR_CONCURRENT_STACKS", "0") == "1":
            return False
        if ops.key_split_parts(dtype=dtype, batch=1, lq=La, heads=pg.heads, l0=La, l1=0, mask_mode=0) != 1:
            return False
        return (ops.pair_eligible(dtype, La, pg.head_dim, runtime.key_norm_bound(pg)) and
                ops.pair_eligible(dtype, n_sub // 64 * 64, pr.head_dim, runtime.key_norm_bound(pr)))

    @staticmethod
    def _split_reloc(dtype, rows: int, n_sub: int) -> bool:
        """The reloc attention as two passes (bf16, a query set that fills the chip without key
        splitting; SR_RELOC_SPLIT=0 turns it off): the shared subsample's whole tiles over all query
        rows on the hand-scheduled sweep, then the own-frame pass whose epilogue folds the first in
        (sr_attn_desc.merge_o).  Measured (one box, kbench): 1.505 + 0.332 = 1.837 ms against 1.883 ms
        in one launch; whole C3 step 417.8 / 418.2 vs 419.5 / 418.9 ms (interleaved).  With a separate
        merge launch instead (round 3, first form) it was break-even."""
        return (os.environ.get("SR_RELOC_SPLIT", "1") == "1" and dtype == torch.bfloat16 and
                (rows + 255) // 256 * 16 >= _RELOC_SPLIT_MIN_WG and n_sub >= 64)

    def _stream2(self, dev):
        """Second HIP stream of the frame-sharded reloc attention (SR_SHARD_CONCURRENT=1)."""
        s = getattr(self, "_shard_side", None)
        if s is None or s.device != torch.device(dev):
            s = torch.cuda.Stream(device=dev)
            self._shard_side = s
        return s

    def _side_stream(self, dev):
        """Second HIP stream for the concurrent reloc block (opt-in: SR_CONCURRENT_STACKS=1)."""
        if os.environ.get("SR_CONCURRENT_STACKS", "0") != "1":
            return None
        s = getattr(self, "_side", None)
        if s is None or s.device != torch.device(dev):
            s = torch.cuda.Stream(device=dev)
            self._side = s
        return s

    def _kv_gemm(self, pb, xn, out, rope, pos):
        """K/V-only projection (qkv weight rows C..3C) with k-norm + RoPE on the K half."""
        C = pb.dim
        epi = runtime.qkv_params(pb, rope, **pos)
        if epi is None:
            ops.gemm(xn, pb.w_qkv[C:], out, _lib.SR_EPI_BIAS, bias=_sl(pb.b_qkv, C, 3 * C), tag="gemm")
        else:
            epi["col_offset"] = C
            ops.gemm(xn, pb.w_qkv[C:], out, _lib.SR_EPI_QKV, bias=_sl(pb.b_qkv, C, 3 * C), qkv=epi, tag="gemm")


# SR_SHARD_TAIL=1 (opt-in): the frame-sharded global block's key-split passes declare their chunk
# tails readable (kv_loc / kv_all are Workspace buffers with 64 padding rows), which sends them to the
# hand-scheduled sweep's ragged variant (round 3 measured it level with the compiled sweep per rank:
# DESIGN.md section 5)
_SHARD_TAIL = os.environ.get("SR_SHARD_TAIL", "0") == "1"
# SR_SHARD_CONCURRENT (default 1; 0 for the A/B): under frame sharding with grouped tails, the reloc
# attention on a second stream beside the global attention.  Rank-0 rehearsal, one box, 2 runs each
# (profiles/r05_j10_rs_*.log): G = 8 69.03 / 69.15 -> 66.87 / 66.98 ms, G = 4 121.8 / 121.0 -> 120.9 /
# 120.7 ms; the sharded GPU tests pass with it
_SHARD_CONCURRENT = os.environ.get("SR_SHARD_CONCURRENT", "1") != "0"
# smallest query set (in 256-row x head workgroups) whose reloc attention runs split (A/B switch)
_RELOC_SPLIT_MIN_WG = int(os.environ.get("SR_RELOC_SPLIT_MIN_WG", "2048"))


def _sl(t, a, b):
    return None if t is None else t[a:b]


def _qs(pb) -> bool:
    """Whether pb's QKV GEMMs here write c*q (runtime.q_prescale): the attention takes q_scaled."""
    return runtime.q_prescale(pb) > 0


def _wait(works):
    for w in works:
        w.wait()
    works.clear()


def shard_range(n: int, G: int, r: int) -> Tuple[int, int]:
    """(start, count) of rank r's contiguous share of n frames over G ranks: the first n % G
    ranks own one frame more than the rest (counts differ by at most one)."""
    base, extra = divmod(n, G)
    return r * base + min(r, extra), base + (1 if r < extra else 0)


def gather_rows(dst: torch.Tensor, src: torch.Tensor, counts: List[int], group, rank: int) -> list:
    """Async gather of every rank's ``src`` rows into ``dst`` = [rank 0's rows ; rank 1's ; ...]
    (``counts[j]`` rows from rank j; row-contiguous tensors).  Equal counts: one
    all_gather_into_tensor (RCCL ring over xGMI).  Uneven counts: one broadcast per non-empty
    rank straight into that rank's slot of ``dst`` — the rows land compact, so no padding row
    can reach a softmax.  Returns the works to wait on."""
    dist = torch.distributed
    if isinstance(group, RankSim):  # no peers: this rank's rows land in its slot, the others stay as they are
        off = sum(counts[:rank])
        dst[off:off + counts[rank]].copy_(src)
        return []
    if len(set(counts)) == 1:
        return [dist.all_gather_into_tensor(dst, src, group=group, async_op=True)]
    offs = np.concatenate([[0], np.cumsum(counts)]).tolist()
    if counts[rank]:
        dst[offs[rank]:offs[rank + 1]].copy_(src)
    return [dist.broadcast(dst[offs[j]:offs[j + 1]], src=dist.get_global_rank(group, j), group=group, async_op=True)
            for j in range(len(counts)) if counts[j]]


class RankSim:
    """Stand-in process group for ONE rank of a ``world``-rank frame-sharded forward, run alone on
    one GPU (``Aggregator.set_frame_sharding(RankSim(8, 0))``): the rank computes exactly its
    share -- its frames' DINO / frame / MLP work, the global block's local and remote attention
    passes over every anchor's keys, the reloc block against the whole anchor subsample, the
    replicated camera head -- but the gathers move nothing (the peers' slots of the gathered K/V
    buffers keep whatever they hold).  Its outputs are therefore NOT the model's; it exists to time
    a rank's step and host submit cost before a multi-GPU run (tools/rank_sim.py)."""

    def __init__(self, world: int, rank: int):
        if not 0 <= rank < world:
            raise ValueError(f"rank {rank} outside a world of {world}")
        self.world, self.rank = int(world), int(rank)

