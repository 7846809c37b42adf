"""Mlp mirror (reference: sailrecon/layers/mlp.py:16-40).

Holds fc1 / fc2 with the reference names.  Inside a Block the forward is part of
``runtime.run_block``; a standalone ``Mlp.forward(x)`` (mlp.py:34-40) is the same two HIP GEMMs:
fc1 with the fused bias + erf-GELU epilogue, fc2 with a bias epilogue (bf16 under autocast,
exact fp32 otherwise).
"""

from typing import Optional

import torch
from torch import Tensor, nn

from .. import _lib, ops, runtime


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
        self._packed = {}

    def _load_from_state_dict(self, *args, **kwargs):
        self._packed.clear()
        return super()._load_from_state_dict(*args, **kwargs)

    def _pack(self, dtype):
        if dtype not in self._packed:
            def w(lin):  # rows padded to the GEMM's 128-column tile (extra outputs are dropped)
                n = lin.weight.shape[0]
                npad = -(-n // 128) * 128
                wt = torch.zeros(npad, lin.weight.shape[1], device=lin.weight.device, dtype=dtype)
                wt[:n] = lin.weight.detach().to(dtype)
                b = None
                if lin.bias is not None:
                    b = torch.zeros(npad, device=lin.weight.device, dtype=torch.float32)
                    b[:n] = lin.bias.detach().float()
                return wt, b, n
            self._packed[dtype] = (w(self.fc1), w(self.fc2))
        return self._packed[dtype]

    def forward(self, x: Tensor) -> Tensor:
        runtime.require_device(x, "Mlp")
        if not (isinstance(self.act, nn.GELU) and self.act.approximate == "none"):
            raise NotImplementedError("Mlp.forward: the fused epilogue is the exact erf GELU (block.py:39)")
        if self.training and self.drop.p > 0:
            raise NotImplementedError("Mlp dropout")
        dtype = runtime.compute_dtype()
        (w1, b1, n1), (w2, b2, n2) = self._pack(dtype)
        kt = 64 if dtype == torch.bfloat16 else 32
        if w1.shape[1] % kt or n1 % kt:
            raise NotImplementedError(f"Mlp.forward: in / hidden features must be multiples of {kt}")
        lead = x.shape[:-1]
        xa = x.detach().reshape(-1, x.shape[-1]).to(dtype).contiguous()
        M = xa.shape[0]
        h = torch.empty(M, w1.shape[0], device=x.device, dtype=dtype)
        ops.gemm(xa, w1, h, _lib.SR_EPI_BIAS_GELU, bias=b1)
        out = torch.empty(M, w2.shape[0], device=x.device, dtype=dtype)
        ops.gemm(h[:, :n1], w2[:, :n1], out, _lib.SR_EPI_BIAS, bias=b2)
        return out[:, :n2].reshape(*lead, n2)
