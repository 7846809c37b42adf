"""Attention mirror (reference: sailrecon/layers/attention.py:21-143).

Names and shapes match the reference state_dict (qkv, q_norm, k_norm, proj).  Inside a Block
the math runs as part of ``runtime.run_block`` (SR_EPI_QKV GEMM with bias + qk-LayerNorm + RoPE
fused -> sr_attention -> proj GEMM with LayerScale and the residual add fused).  A standalone
``Attention.forward(x, pos, attn_mask)`` (attention.py:70-122) runs the same kernels with a plain
bias epilogue on proj: bf16 under autocast (the reference's autocast Linear returns bf16), exact
fp32 otherwise.  ``attn_mask``: anything F.scaled_dot_product_attention accepts — a bool mask
(True = attend) or a float mask added to the scores, broadcastable to [B, heads, N, N] — runs on
the exact fp32 kernel with the mask read in place (SR_MASK_DENSE / SR_MASK_ADD; broadcast dims
keep stride 0, nothing is expanded in memory and nothing is inspected on the host).
"""

from __future__ import annotations

from typing import Optional, Tuple

import torch
from torch import Tensor, nn

from .. import _lib, ops, runtime


def sdpa_mask(attn_mask: Tensor, B: int, heads: int, N: int, L: int, device) -> Tuple[int, Tensor]:
    """(mask_mode, [B, heads, N, L] view) for ops.attention from an SDPA ``attn_mask``
    (attention.py:103-109): bool -> SR_MASK_DENSE (True = attend), floating -> SR_MASK_ADD (fp32,
    added to the scaled scores).  Broadcast dims stay stride 0; only a mask whose key dim is not
    unit-stride is copied."""
    if attn_mask.dim() > 4:
        raise ValueError(f"attn_mask of rank {attn_mask.dim()} cannot broadcast to [B, heads, N, N]")
    m = attn_mask.to(device)
    if m.dtype == torch.bool:
        mode = _lib.SR_MASK_DENSE
    elif m.is_floating_point():
        mode = _lib.SR_MASK_ADD
        m = m.float()
    else:
        raise TypeError(f"attn_mask must be bool or floating (got {m.dtype})")
    m = m.expand(B, heads, N, L)
    if m.stride(3) != 1:
        m = m.contiguous()
    return mode, m


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
        self._packed = {}

    def clear_kv_cache(self):
        self.k_cache = None
        self.v_cache = None

    def _load_from_state_dict(self, *args, **kwargs):
        self._packed.clear()
        return super()._load_from_state_dict(*args, **kwargs)

    def packed(self, dtype: torch.dtype) -> runtime.PackedBlock:
        if dtype not in self._packed:
            self._packed[dtype] = runtime.pack_attention(self, dtype)
        return self._packed[dtype]

    def forward(self, x: Tensor, pos: Optional[Tensor] = None, attn_mask: Optional[Tensor] = None) -> Tensor:
        runtime.require_device(x, "Attention")
        if self.kv_cache:
            raise NotImplementedError("the kv-cache attention (attention.py:85-100) runs inside "
                                      "Aggregator.forward / forward_with_cache (SailRecon.tmp_forward / reloc)")
        if self.training and self.attn_drop.p > 0:
            raise NotImplementedError("attention dropout")
        B, N, C = x.shape
        dtype = runtime.compute_dtype()
        if attn_mask is not None or self.head_dim != 64:
            dtype = torch.float32  # the MFMA attention kernel is head_dim 64, unmasked
        pa = self.packed(dtype)
        xa = x.detach().reshape(B * N, C).to(dtype).contiguous()
        qkv = torch.empty(B * N, 3 * C, device=x.device, dtype=dtype)
        if self.rope is not None and pos is not None:
            rope = self.rope.tables(self.head_dim, int(pos.max()) + 1, x.device)
            pos_yx = pos.reshape(B * N, 2).to(device=x.device, dtype=torch.int32).contiguous()
            epi = runtime.qkv_params(pa, rope, prescale=True, pos_yx=pos_yx)
        else:
            epi = runtime.qkv_params(pa, None, prescale=True)
        qs = runtime.q_prescale(pa)  # bf16: c*q rounded once by the GEMM (0 in fp32 mode)
        runtime.qkv_gemm(pa, xa, pa.w_qkv, qkv, pa.b_qkv, epi, qs)
        o = torch.empty(B * N, C, device=x.device, dtype=dtype)
        if attn_mask is None:
            runtime.frame_attend(pa, B, N, q_scaled=qs > 0)(qkv, o)
        else:
            mode, m = sdpa_mask(attn_mask, B, self.num_heads, N, N, x.device)
            ops.attention(qkv[:, 0:C], qkv[:, C:2 * C], qkv[:, 2 * C:], o, heads=self.num_heads,
                          head_dim=self.head_dim, batch=B, lq=N, q_bstride=N, l0=N, k0_bstride=N,
                          mask_mode=mode, mask=m)
        out = torch.empty(B * N, C, device=x.device, dtype=dtype)
        ops.gemm(o, pa.w_proj, out, _lib.SR_EPI_BIAS, bias=pa.b_proj)
        return out.view(B, N, C)


class MemEffAttention(Attention):
    """DINOv2 attention class (attention.py:125-143); identical parameters.  Without xFormers the
    reference asserts ``pos is None`` and ``attn_bias is None`` and falls back to Attention."""

    def forward(self, x: Tensor, attn_bias=None, pos=None, attn_mask=None) -> Tensor:
        assert pos is None
        if attn_bias is not None:
            raise AssertionError("xFormers is required for using nested tensors")
        return super().forward(x, attn_mask=attn_mask)
