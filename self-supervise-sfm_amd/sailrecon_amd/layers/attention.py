"""Attention mirror (reference: sailrecon/layers/attention.py:21-143).

Names and shapes match the reference state_dict (qkv, q_norm, k_norm, proj).  Inside a Block
the math runs as part of ``runtime.run_block`` (SR_EPI_QKV GEMM with bias + qk-LayerNorm + RoPE
fused -> sr_attention -> proj GEMM with LayerScale and the residual add fused).  A standalone
``Attention.forward(x, pos, attn_mask)`` (attention.py:70-122) runs the same kernels with a plain
bias epilogue on proj: bf16 under autocast (the reference's autocast Linear returns bf16), exact
fp32 otherwise.  Masks: None, or the camera-trunk pattern (camera_head.py:197-228), as Block.
"""

from __future__ import annotations

from typing import Optional

import torch
from torch import Tensor, nn

from .. import _lib, ops, runtime


def camera_mask_anchors(attn_mask: Tensor) -> Optional[int]:
    """If ``attn_mask`` (True = attend, [1,1,S,S] or [S,S]) is the camera-trunk pattern,
    return its anchor count; else None."""
    m = attn_mask.reshape(attn_mask.shape[-2], attn_mask.shape[-1]).bool().cpu()
    S = m.shape[0]
    for n in range(1, S + 1):
        ref = torch.zeros(S, S, dtype=torch.bool)
        ref[:, :n] = True
        idx = torch.arange(n, S)
        ref[:n, n:] = False
        ref[idx, idx] = True
        if torch.equal(ref, m):
            return n
    return None


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
        n_anchor = None
        if attn_mask is not None:
            n_anchor = camera_mask_anchors(attn_mask)
            if n_anchor is None:
                raise NotImplementedError("Attention.forward: only None or the camera-trunk mask is supported "
                                          "(the aggregator drives the reloc block mask implicitly)")
            if B != 1:
                raise NotImplementedError("Attention.forward: masked attention needs B == 1")
        if n_anchor is not None or self.head_dim != 64:
            dtype = torch.float32  # the MFMA attention kernel is head_dim 64, unmasked
        pa = self.packed(dtype)
        xa = x.detach().reshape(B * N, C).to(dtype).contiguous()
        qkv = torch.empty(B * N, 3 * C, device=x.device, dtype=dtype)
        if self.rope is not None and pos is not None:
            rope = self.rope.tables(self.head_dim, int(pos.max()) + 1, x.device)
            pos_yx = pos.reshape(B * N, 2).to(device=x.device, dtype=torch.int32).contiguous()
            epi = runtime.qkv_params(pa, rope, pos_yx=pos_yx)
        else:
            epi = runtime.qkv_params(pa, None)
        if epi is None:
            ops.gemm(xa, pa.w_qkv, qkv, _lib.SR_EPI_BIAS, bias=pa.b_qkv)
        else:
            ops.gemm(xa, pa.w_qkv, qkv, _lib.SR_EPI_QKV, bias=pa.b_qkv, qkv=epi)
        o = torch.empty(B * N, C, device=x.device, dtype=dtype)
        if n_anchor is None:
            runtime.frame_attend(pa, B, N)(qkv, o)
        else:
            ops.attention(qkv[:, 0:C], qkv[:, C:2 * C], qkv[:, 2 * C:], o, heads=self.num_heads,
                          head_dim=self.head_dim, batch=1, lq=N, q_bstride=0, l0=N, k0_bstride=0,
                          mask_mode=_lib.SR_MASK_CAMERA, n_anchor=n_anchor)
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
