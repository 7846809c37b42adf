"""LayerScale mirror (reference: sailrecon/layers/layer_scale.py:14-23).

Inside a Block gamma is applied in the residual GEMM epilogue (SR_EPI_BIAS_RESID); a standalone
``LayerScale.forward(x)`` is the sr_mul_cols kernel (x * gamma per column, in place when
``inplace`` as the reference's ``x.mul_``).
"""

import torch
from torch import Tensor, nn

from .. import ops, runtime


class LayerScale(nn.Module):
    def __init__(self, dim: int, init_values: float = 1e-5, inplace: bool = False) -> None:
        super().__init__()
        self.inplace = inplace
        self.gamma = nn.Parameter(init_values * torch.ones(dim))

    def forward(self, x: Tensor) -> Tensor:
        runtime.require_device(x, "LayerScale")
        if x.dtype not in (torch.float32, torch.bfloat16) or not x.is_contiguous():
            raise NotImplementedError("LayerScale.forward: contiguous fp32 / bf16 input")
        x2 = x.view(-1, x.shape[-1])
        out = x2 if self.inplace else torch.empty_like(x2)
        ops.mul_cols(x2, self.gamma.detach().float().contiguous(), out)
        return x if self.inplace else out.view(x.shape)
