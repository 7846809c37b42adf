"""DINOv2 ViT parameter mirror (reference: sailrecon/layers/vision_transformer.py:53-443).

Same parameter names / shapes (``cls_token``, ``pos_embed``, ``register_tokens``,
``mask_token``, ``patch_embed.proj``, ``blocks.#``, ``norm``).  Its forward is driven
by the aggregator engine (``models/aggregator.py``): im2col + patch GEMM with the
positional add fused, 24 frame-local Blocks, final LayerNorm (eps 1e-6).
"""

from __future__ import annotations

import math
from functools import partial

import torch
import torch.nn.functional as F
from torch import nn

from .attention import MemEffAttention
from .block import NestedTensorBlock as Block
from .mlp import Mlp
from .patch_embed import PatchEmbed


class DinoVisionTransformer(nn.Module):
    def __init__(self, img_size=224, patch_size=16, in_chans=3, embed_dim=768, depth=12, num_heads=12,
                 mlp_ratio=4.0, qkv_bias=True, ffn_bias=True, proj_bias=True, drop_path_rate=0.0,
                 drop_path_uniform=False, init_values=None, embed_layer=PatchEmbed, act_layer=nn.GELU,
                 block_fn=Block, ffn_layer="mlp", block_chunks=1, num_register_tokens=0,
                 interpolate_antialias=False, interpolate_offset=0.1, qk_norm=False):
        super().__init__()
        if ffn_layer != "mlp":
            raise NotImplementedError("only the Mlp FFN is on the SailRecon path (vision_transformer.py:145-147)")
        if block_chunks not in (0, 1) and block_chunks is not None:
            raise NotImplementedError("block_chunks > 1 is not used by the aggregator (aggregator.py:204)")
        norm_layer = partial(nn.LayerNorm, eps=1e-6)
        self.num_features = self.embed_dim = embed_dim
        self.num_tokens = 1
        self.n_blocks = depth
        self.num_heads = num_heads
        self.patch_size = patch_size
        self.num_register_tokens = num_register_tokens
        self.interpolate_antialias = interpolate_antialias
        self.interpolate_offset = interpolate_offset
        self.patch_embed = embed_layer(img_size=img_size, patch_size=patch_size, in_chans=in_chans,
                                       embed_dim=embed_dim)
        num_patches = self.patch_embed.num_patches
        self.cls_token = nn.Parameter(torch.zeros(1, 1, embed_dim))
        self.pos_embed = nn.Parameter(torch.zeros(1, num_patches + self.num_tokens, embed_dim))
        self.register_tokens = (nn.Parameter(torch.zeros(1, num_register_tokens, embed_dim))
                                if num_register_tokens else None)
        self.chunked_blocks = False
        self.blocks = nn.ModuleList([
            block_fn(dim=embed_dim, num_heads=num_heads, mlp_ratio=mlp_ratio, qkv_bias=qkv_bias,
                     proj_bias=proj_bias, ffn_bias=ffn_bias, drop_path=0.0, norm_layer=norm_layer,
                     act_layer=act_layer, ffn_layer=Mlp, init_values=init_values, qk_norm=qk_norm)
            for _ in range(depth)
        ])
        self.norm = norm_layer(embed_dim)
        self.head = nn.Identity()
        self.mask_token = nn.Parameter(torch.zeros(1, embed_dim))
        nn.init.trunc_normal_(self.pos_embed, std=0.02)
        nn.init.normal_(self.cls_token, std=1e-6)
        if self.register_tokens is not None:
            nn.init.normal_(self.register_tokens, std=1e-6)
        self._pos_cache = {}

    def pos_embed_for(self, h_img: int, w_img: int) -> torch.Tensor:
        """[1 + npatch, C] fp32 positional table for an h_img x w_img input.

        interpolate_pos_encoding, vision_transformer.py:206-240: returned as-is when the
        patch count matches and the image is square; otherwise bicubic (antialias per
        ctor) resampling of the patch part.  Parameter preprocessing, computed once per
        resolution and cached on the device.
        """
        npatch = (h_img // self.patch_size) * (w_img // self.patch_size)
        key = (h_img, w_img, self.pos_embed.device, self.pos_embed._version)
        if key in self._pos_cache:
            return self._pos_cache[key]
        pe = self.pos_embed.detach()
        if not self.pos_resampled(h_img, w_img):
            out = pe[0].float().contiguous()
        else:
            # bicubic resampling of a parameter table (not a per-forward op): run on the host
            pe = pe.float()
            pp = self.resample_patch_pos(pe[0, 1:].cpu(), h_img, w_img)
            out = torch.cat([pe[0, :1].cpu(), pp], dim=0).to(pe.device).contiguous()
        self._pos_cache = {key: out}
        return out

    def pos_resampled(self, h_img: int, w_img: int) -> bool:
        npatch = (h_img // self.patch_size) * (w_img // self.patch_size)
        return not (npatch == self.pos_embed.shape[1] - 1 and w_img == h_img)

    def resample_patch_pos(self, patch_pe: torch.Tensor, h_img: int, w_img: int) -> torch.Tensor:
        """[n0, C] patch part of pos_embed -> [npatch, C] for an h_img x w_img input: the bicubic
        resampling of interpolate_pos_encoding (vision_transformer.py:219-238).  Linear in
        ``patch_pe``, so the training backward takes its adjoint by autograd (TrainGraph)."""
        n0, dim = patch_pe.shape
        m = int(math.sqrt(n0))
        assert n0 == m * m
        kw = {}
        if self.interpolate_offset:
            kw["scale_factor"] = (float(h_img // self.patch_size + self.interpolate_offset) / m,
                                  float(w_img // self.patch_size + self.interpolate_offset) / m)
        else:
            kw["size"] = (h_img // self.patch_size, w_img // self.patch_size)
        src = patch_pe.reshape(1, m, m, dim).permute(0, 3, 1, 2)
        pp = F.interpolate(src, mode="bicubic", antialias=self.interpolate_antialias, **kw)
        return pp.permute(0, 2, 3, 1).reshape(-1, dim)


def vit_small(patch_size=16, num_register_tokens=0, **kwargs):
    return DinoVisionTransformer(patch_size=patch_size, embed_dim=384, depth=12, num_heads=6, mlp_ratio=4,
                                 block_fn=partial(Block, attn_class=MemEffAttention),
                                 num_register_tokens=num_register_tokens, **kwargs)


def vit_base(patch_size=16, num_register_tokens=0, **kwargs):
    return DinoVisionTransformer(patch_size=patch_size, embed_dim=768, depth=12, num_heads=12, mlp_ratio=4,
                                 block_fn=partial(Block, attn_class=MemEffAttention),
                                 num_register_tokens=num_register_tokens, **kwargs)


def vit_large(patch_size=16, num_register_tokens=0, **kwargs):
    return DinoVisionTransformer(patch_size=patch_size, embed_dim=1024, depth=24, num_heads=16, mlp_ratio=4,
                                 block_fn=partial(Block, attn_class=MemEffAttention),
                                 num_register_tokens=num_register_tokens, **kwargs)


def vit_giant2(patch_size=16, num_register_tokens=0, **kwargs):
    return DinoVisionTransformer(patch_size=patch_size, embed_dim=1536, depth=40, num_heads=24, mlp_ratio=4,
                                 block_fn=partial(Block, attn_class=MemEffAttention),
                                 num_register_tokens=num_register_tokens, **kwargs)
