"""Mlp parameter mirror (reference: sailrecon/layers/mlp.py:16-40).

Holds fc1 / fc2 with the reference names; the forward runs on the HIP path as
GEMM(fc1, fused bias + erf-GELU) -> GEMM(fc2) inside ``runtime.run_block``.
"""

from typing import Optional

from torch import nn


class Mlp(nn.Module):
    def __init__(self, in_features: int, hidden_features: Optional[int] = None,
                 out_features: Optional[int] = None, act_layer=nn.GELU, drop: float = 0.0,
                 bias: bool = True) -> None:
        super().__init__()
        out_features = out_features or in_features
        hidden_features = hidden_features or in_features
        self.fc1 = nn.Linear(in_features, hidden_features, bias=bias)
        self.act = act_layer()
        self.fc2 = nn.Linear(hidden_features, out_features, bias=bias)
        self.drop = nn.Dropout(drop)
