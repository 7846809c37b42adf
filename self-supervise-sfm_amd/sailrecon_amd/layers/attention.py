"""Attention parameter mirror (reference: sailrecon/layers/attention.py:21-143).

Names and shapes match the reference state_dict (qkv, q_norm, k_norm, proj).  The
math runs on the HIP path: SR_EPI_QKV GEMM (bias + qk-LayerNorm + RoPE fused) ->
sr_attention -> SR_EPI_BIAS_RESID GEMM, see ``runtime.run_block``.
"""

from torch import nn


class Attention(nn.Module):
    def __init__(self, dim: int, num_heads: int = 8, qkv_bias: bool = True, proj_bias: bool = True,
                 attn_drop: float = 0.0, proj_drop: float = 0.0, norm_layer=nn.LayerNorm, qk_norm: bool = False,
                 fused_attn: bool = True, rope=None, kv_cache: bool = False) -> None:
        super().__init__()
        assert dim % num_heads == 0, "dim should be divisible by num_heads"
        self.num_heads = num_heads
        self.head_dim = dim // num_heads
        self.scale = self.head_dim ** -0.5
        self.fused_attn = fused_attn
        self.kv_cache = kv_cache
        self.k_cache = None
        self.v_cache = None
        self.qkv = nn.Linear(dim, dim * 3, bias=qkv_bias)
        self.q_norm = norm_layer(self.head_dim) if qk_norm else nn.Identity()
        self.k_norm = norm_layer(self.head_dim) if qk_norm else nn.Identity()
        self.attn_drop = nn.Dropout(attn_drop)
        self.proj = nn.Linear(dim, dim, bias=proj_bias)
        self.proj_drop = nn.Dropout(proj_drop)
        self.rope = rope
        self.qk_norm = qk_norm

    def clear_kv_cache(self):
        self.k_cache = None
        self.v_cache = None


class MemEffAttention(Attention):
    """DINOv2 attention class (attention.py:125-143); identical parameters."""
