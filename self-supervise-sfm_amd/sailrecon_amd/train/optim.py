"""Optimizer side of the training step (train_imc.py:476-497, 404-411), over FlatParams:

  Adam                  torch.optim.Adam(lr, betas=(0.9, 0.999), eps=1e-8) semantics; one
                        sr_adam_f32 launch over the flat fp32 buffer (parameters whose grad
                        stays zero, e.g. the DPT heads that no loss reaches, are left unchanged:
                        m = v = 0 gives a zero update, as torch skips grad-less params)
  GradScaler            torch.cuda.amp.GradScaler defaults (init 2^16, growth 2, backoff 0.5,
                        interval 2000): the loss seed is scaled, the inf/nan check runs on the
                        device (sr_nonfinite_check), Adam unscales and skips on inf
  CosineWarmupScheduler train_imc.py:62-86, verbatim semantics (host scalar)
"""

from __future__ import annotations

import math
from typing import Optional

import torch

from .. import ops
from .params import FlatParams


class Adam:
    def __init__(self, flat: FlatParams, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0):
        self.flat = flat
        self.param_groups = [dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay)]
        self.m = torch.zeros_like(flat.data)
        self.v = torch.zeros_like(flat.data)
        self.step_count = 0

    def zero_grad(self) -> None:
        self.flat.zero_grad()

    def step(self, scale: Optional[torch.Tensor] = None, found_inf: Optional[torch.Tensor] = None) -> None:
        """One Adam step; ``scale`` (device [1]) divides the gradients first (GradScaler.unscale_
        and the data-parallel mean), ``found_inf`` (device int [1]) skips the update."""
        g = self.param_groups[0]
        self.step_count += 1
        ops.adam(self.flat.data, self.flat.grad, self.m, self.v, lr=g["lr"], beta1=g["betas"][0], beta2=g["betas"][1],
                 eps=g["eps"], weight_decay=g["weight_decay"], step=self.step_count, scale=scale, found_inf=found_inf)


class GradScaler:
    def __init__(self, init_scale: float = 2.0 ** 16, growth_factor: float = 2.0, backoff_factor: float = 0.5,
                 growth_interval: int = 2000, enabled: bool = True):
        self.enabled = enabled
        self._scale = init_scale if enabled else 1.0
        self.growth_factor, self.backoff_factor, self.growth_interval = growth_factor, backoff_factor, growth_interval
        self._growth_tracker = 0
        self._dev = {}

    def get_scale(self) -> float:
        return self._scale

    def _buffers(self, device):
        key = str(device)
        if key not in self._dev:
            self._dev[key] = (torch.zeros(1, device=device, dtype=torch.float32),
                              torch.zeros(1, device=device, dtype=torch.int32))
        return self._dev[key]

    def step(self, optimizer: Adam, world_size: int = 1, before_sync=None) -> bool:
        """unscale (by scale * world_size: DDP's mean), check, step unless inf; returns found_inf
        (reads one int back: the reference reads loss.item() every step anyway).  ``before_sync``:
        called after the update is queued and before that read, so that its launches (the weight
        refresh) keep the GPU busy while the host waits (a skipped update leaves the weights, so
        work derived from them comes out the same)."""
        dev = optimizer.flat.grad.device
        scale_t, found = self._buffers(dev)
        scale_t.fill_(self._scale * world_size)
        if not self.enabled:
            # a disabled torch GradScaler steps unconditionally: no inf/NaN check, no skip
            optimizer.step(scale=scale_t, found_inf=None)
            if before_sync is not None:
                before_sync()
            self._found = False
            return False
        found.zero_()
        ops.nonfinite_check(optimizer.flat.grad, found, scale_t)
        optimizer.step(scale=scale_t, found_inf=found)
        if before_sync is not None:
            before_sync()
        self._found = bool(found.item())
        if self._found:
            optimizer.step_count -= 1  # torch.optim.Adam's state step does not advance on a skipped step
        return self._found

    def update(self) -> None:
        if not self.enabled:
            return
        if getattr(self, "_found", False):
            self._scale *= self.backoff_factor
            self._growth_tracker = 0
        else:
            self._growth_tracker += 1
            if self._growth_tracker == self.growth_interval:
                self._scale *= self.growth_factor
                self._growth_tracker = 0


class CosineWarmupScheduler:
    def __init__(self, optimizer, warmup_steps, max_steps, max_lr, min_lr=0):
        self.optimizer = optimizer
        self.warmup_steps = warmup_steps
        self.max_steps = max_steps
        self.max_lr = max_lr
        self.min_lr = min_lr
        self.step_count = 0

    def step(self) -> float:
        self.step_count += 1
        if self.step_count <= self.warmup_steps:
            lr = self.max_lr * self.step_count / self.warmup_steps
        else:
            progress = (self.step_count - self.warmup_steps) / (self.max_steps - self.warmup_steps)
            lr = self.min_lr + (self.max_lr - self.min_lr) * 0.5 * (1 + math.cos(math.pi * progress))
        for pg in self.optimizer.param_groups:
            pg["lr"] = lr
        return lr
