"""LayerScale parameter mirror (reference: sailrecon/layers/layer_scale.py:14-23).

gamma is applied inside the residual GEMM epilogue (SR_EPI_BIAS_RESID).
"""

import torch
from torch import nn


class LayerScale(nn.Module):
    def __init__(self, dim: int, init_values: float = 1e-5, inplace: bool = False) -> None:
        super().__init__()
        self.inplace = inplace
        self.gamma = nn.Parameter(init_values * torch.ones(dim))
