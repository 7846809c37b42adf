"""Flat fp32 parameter / gradient / optimizer-state buffers (the layout the DDP all-reduce and
the fused Adam step run over; train_imc.py:474-480 wraps the model in DDP + optim.Adam).

Every trainable parameter's ``.data`` and ``.grad`` become views into ONE contiguous fp32
buffer each (offsets aligned to 64 floats = 256 B), in ``named_parameters`` order, so that:
  * one RCCL all-reduce (bucketed over slices) covers every gradient (train.dist);
  * one sr_adam_f32 launch per bucket updates every parameter (train.optim.Adam);
  * q_norm / k_norm weight|bias grads (64 floats each) form the contiguous [4, 64] block the
    qk backward kernel accumulates into.
Parameters with ``requires_grad=False`` (DINO's mask_token, aggregator.py:229) stay outside.
"""

from __future__ import annotations

from typing import Dict, List, Tuple

import torch
from torch import nn

ALIGN = 64


class FlatParams:
    def __init__(self, module: nn.Module, device=None):
        self.names: List[str] = []
        self.offsets: Dict[str, Tuple[int, int]] = {}
        params = [(n, p) for n, p in module.named_parameters() if p.requires_grad]
        off = 0
        for n, p in params:
            self.names.append(n)
            self.offsets[n] = (off, p.numel())
            off += -(-p.numel() // ALIGN) * ALIGN
        self.numel = off
        dev = device if device is not None else (params[0][1].device if params else "cpu")
        self.data = torch.zeros(self.numel, device=dev, dtype=torch.float32)
        self.grad = torch.zeros(self.numel, device=dev, dtype=torch.float32)
        self.params = dict(params)
        for n, p in params:
            o, k = self.offsets[n]
            if p.dtype != torch.float32:
                raise TypeError(f"{n}: training keeps fp32 master parameters (got {p.dtype})")
            self.data[o:o + k].copy_(p.detach().reshape(-1))
            p.data = self.data[o:o + k].view_as(p)
            p.grad = self.grad[o:o + k].view_as(p)

    def zero_grad(self) -> None:
        self.grad.zero_()  # one memset (plumbing)

    def view(self, flat: torch.Tensor, name: str) -> torch.Tensor:
        o, k = self.offsets[name]
        return flat[o:o + k].view_as(self.params[name])
