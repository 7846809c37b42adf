"""2-D RoPE tables and token positions (reference: sailrecon/layers/rope.py).

The rotation itself is fused into the QKV GEMM epilogue (SR_EPI_QKV); this module
only builds the cos/sin tables, computed with the same fp32 torch ops as
rope.py:93-124 so the device path consumes bit-identical angles.  Positions are
derived in-kernel from the token row (PositionGetter, rope.py:40-66, plus the
``pos + 1`` / zero-for-special-tokens rule of aggregator.py:313-328).
"""

from __future__ import annotations

from typing import Dict, Tuple

import torch
from torch import nn


class PositionGetter:
    """rope.py:25-66 — (y, x) grid positions, cached per grid size."""

    def __init__(self):
        self.position_cache: Dict[Tuple[int, int], torch.Tensor] = {}

    def __call__(self, batch_size: int, height: int, width: int, device) -> torch.Tensor:
        if (height, width) not in self.position_cache:
            y = torch.arange(height, device=device)
            x = torch.arange(width, device=device)
            self.position_cache[height, width] = torch.cartesian_prod(y, x)
        pos = self.position_cache[height, width]
        return pos.view(1, height * width, 2).expand(batch_size, -1, -1).clone()


class RotaryPositionEmbedding2D(nn.Module):
    def __init__(self, frequency: float = 100.0, scaling_factor: float = 1.0):
        super().__init__()
        self.base_frequency = frequency
        self.scaling_factor = scaling_factor
        self._tables: Dict[Tuple, Tuple[torch.Tensor, torch.Tensor]] = {}

    def tables(self, head_dim: int, max_pos: int, device) -> Tuple[torch.Tensor, torch.Tensor]:
        """cos/sin [max_pos, head_dim // 4] fp32 for the epilogue (first half of the
        duplicated cat(angles, angles) table; rope.py:119)."""
        key = (head_dim, max_pos, str(device))
        if key not in self._tables:
            dim = head_dim // 2  # per spatial direction (rope.py:187)
            exponents = torch.arange(0, dim, 2).float() / dim
            inv_freq = 1.0 / (self.base_frequency ** exponents)
            positions = torch.arange(max_pos, dtype=inv_freq.dtype)
            angles = torch.einsum("i,j->ij", positions, inv_freq)
            self._tables[key] = (angles.cos().contiguous().to(device), angles.sin().contiguous().to(device))
        return self._tables[key]
