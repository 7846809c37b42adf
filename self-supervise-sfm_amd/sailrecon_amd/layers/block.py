"""Block parameter mirror + standalone device forward (reference: sailrecon/layers/block.py).

``Block.forward(x, pos=None, attn_mask=None)`` keeps the reference signature
(block.py:86).  It runs the whole block on the HIP path (runtime.run_block) for
x on a ROCm device: bf16 under autocast, exact fp32 otherwise.  ``attn_mask`` is
anything F.scaled_dot_product_attention accepts (bool, True = attend, or an additive
float mask, broadcastable to [B, heads, N, N]); a masked block runs the exact fp32
kernel with the mask read in place (layers/attention.py sdpa_mask).  Inside the
model the aggregator drives the reloc block mask and the camera head its trunk mask
implicitly (no mask tensor).
"""

from __future__ import annotations

from typing import Callable, Optional

import torch
from torch import Tensor, nn

from .. import ops, runtime
from .attention import Attention, sdpa_mask
from .layer_scale import LayerScale
from .mlp import Mlp


class Block(nn.Module):
    def __init__(self, dim: int, num_heads: int, mlp_ratio: float = 4.0, qkv_bias: bool = True,
                 proj_bias: bool = True, ffn_bias: bool = True, drop: float = 0.0, attn_drop: float = 0.0,
                 init_values=None, drop_path: float = 0.0, act_layer: Callable[..., nn.Module] = nn.GELU,
                 norm_layer: Callable[..., nn.Module] = nn.LayerNorm, attn_class: Callable[..., nn.Module] = Attention,
                 ffn_layer: Callable[..., nn.Module] = Mlp, qk_norm: bool = False, fused_attn: bool = True,
                 rope=None, kv_cache: bool = False) -> None:
        super().__init__()
        self.norm1 = norm_layer(dim)
        self.attn = attn_class(dim, num_heads=num_heads, qkv_bias=qkv_bias, proj_bias=proj_bias,
                               attn_drop=attn_drop, proj_drop=drop, qk_norm=qk_norm, fused_attn=fused_attn,
                               rope=rope, kv_cache=kv_cache)
        self.ls1 = LayerScale(dim, init_values=init_values) if init_values else nn.Identity()
        self.norm2 = norm_layer(dim)
        self.mlp = ffn_layer(in_features=dim, hidden_features=int(dim * mlp_ratio), act_layer=act_layer, drop=drop,
                             bias=ffn_bias)
        self.ls2 = LayerScale(dim, init_values=init_values) if init_values else nn.Identity()
        self.sample_drop_ratio = drop_path
        self._packed = {}

    def packed(self, dtype: torch.dtype) -> runtime.PackedBlock:
        if dtype not in self._packed:
            self._packed[dtype] = runtime.pack_block(self, dtype)
        return self._packed[dtype]

    def invalidate_packed(self):
        self._packed.clear()

    def forward(self, x: Tensor, pos: Optional[Tensor] = None, attn_mask: Optional[Tensor] = None) -> Tensor:
        runtime.require_device(x, "Block")
        dtype = runtime.compute_dtype()
        B, N, C = x.shape
        pb = self.packed(dtype)
        if attn_mask is not None or pb.head_dim != 64:
            dtype = torch.float32
            pb = self.packed(dtype)
        xf = x.detach().reshape(B * N, C).float().contiguous().clone()
        ws = runtime.Workspace()
        sc = runtime.scratch(ws, B * N, C, pb.w_fc1.shape[0], dtype, x.device)
        rope = None
        qkv_epi = None
        if self.attn.rope is not None and pos is not None:
            rope = self.attn.rope.tables(pb.head_dim, int(pos.max()) + 1, x.device)
            pos_yx = pos.reshape(B * N, 2).to(device=x.device, dtype=torch.int32).contiguous()
            qkv_epi = runtime.qkv_params(pb, rope, prescale=True, pos_yx=pos_yx)
        else:
            qkv_epi = runtime.qkv_params(pb, None, prescale=True)
        qs = runtime.q_prescale(pb)  # bf16: the QKV GEMM writes c*q, rounded once (0 in fp32 mode)
        if attn_mask is None:
            attend = runtime.frame_attend(pb, B, N, q_scaled=qs > 0)
        else:
            mode, m = sdpa_mask(attn_mask, B, pb.heads, N, N, x.device)

            def attend(qkv, o):
                ops.attention(qkv[:, 0:C], qkv[:, C:2 * C], qkv[:, 2 * C:], o, heads=pb.heads, head_dim=pb.head_dim,
                              batch=B, lq=N, q_bstride=N, l0=N, k0_bstride=N, mask_mode=mode, mask=m)
        runtime.run_block(pb, xf, 0, B * N, sc, attend, qkv_epi, q_scale=qs)
        return xf.view(B, N, C).to(x.dtype)


class NestedTensorBlock(Block):
    """DINOv2 block class name (block.py:271); tensors only (no xFormers nesting)."""
