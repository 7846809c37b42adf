"""One self-supervised training step on the HIP path — train_epoch's loop body
(train/train_imc.py:366-411) for SailRecon under DDP (train_imc.py:474-480):

    optimizer.zero_grad()
    predictions = model.forward(duplicated_images, no_reloc_list, reloc_list)   (bf16 autocast)
    loss = compute_loss(predictions, batch, ...)                                   (fp32)
    scaler.scale(loss).backward();  scaler.step(optimizer);  scaler.update();  scheduler.step()

Data parallel: one process per GPU, one scene per rank; gradients are averaged over the ranks
with torch.distributed all-reduces (RCCL over xGMI with the "nccl" backend) issued per module as
soon as the backward has finished it (TrainGraph.grad_ready_hook) so they overlap the rest of the
backward — the role of DDP's gradient buckets.  Parameters no loss reaches (the DPT heads) keep
zero grads on every rank and are not reduced (their mean is zero either way).
"""

from __future__ import annotations

from pathlib import Path
from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist

from .loss import CDFLossIndexPytorch, imc_loss
from .model import TrainGraph
from .optim import Adam, CosineWarmupScheduler, GradScaler

Tensor = torch.Tensor


def prepare_model_input(rgb: Tensor) -> Tuple[Tensor, List[int], List[int]]:
    """train_imc.py:107-138: duplicate the N views (anchors, then the same images as queries)."""
    n = rgb.shape[0]
    return torch.cat([rgb, rgb], 0)[None], list(range(n)), list(range(n, 2 * n))


def save_checkpoint(model, optimizer, scheduler, scaler, step: int, loss, checkpoint_dir,
                    is_distributed: bool = False) -> Path:
    """train_imc.py:272-286: model weights only, as ``model_step_<step>.pt`` and ``model_latest.pt``
    (a plain state_dict with the reference's keys, so the reference's own loader and
    ``SailRecon.load_state_dict`` both read it).  The trainer's parameters are views into its flat
    fp32 buffer (train.params.FlatParams), so ``state_dict()`` already holds the updated weights.
    ``optimizer`` / ``scheduler`` / ``scaler`` / ``loss`` are accepted and unused, as in the reference."""
    del optimizer, scheduler, scaler, loss
    checkpoint_dir = Path(checkpoint_dir)
    checkpoint_dir.mkdir(parents=True, exist_ok=True)
    sd = model.module.state_dict() if is_distributed else model.state_dict()
    path = checkpoint_dir / f"model_step_{step}.pt"
    torch.save(sd, path)
    torch.save(sd, checkpoint_dir / "model_latest.pt")
    return path


class Trainer:
    def __init__(self, model, *, max_lr: float = 2e-4, warmup_steps: int = 2000, max_steps: int = 100_000,
                 group=None, grad_scaler: bool = True, cdf: Optional[CDFLossIndexPytorch] = None):
        self.graph = TrainGraph(model)
        self.flat = self.graph.flat
        self.opt = Adam(self.flat, lr=max_lr, betas=(0.9, 0.999), eps=1e-8)           # train_imc.py:480
        self.sched = CosineWarmupScheduler(self.opt, warmup_steps, max_steps, max_lr, max_lr * 0.01)
        self.scaler = GradScaler(enabled=grad_scaler)
        # train_epoch's module (train_imc.py:334-350): dummy single-entry indices -> one histogram
        self.cdf = cdf if cdf is not None else CDFLossIndexPytorch(0.0, 15.0, 250, torch.tensor([0]),
                                                                   torch.tensor([0]), gradient_smooth=0.05)
        self.group = group
        self.world = dist.get_world_size(group) if group is not None else 1
        self._works = []
        self.steps_done = 0
        self._reduced: Dict[int, Tuple[int, int]] = {}
        self._slices = self._module_slices(model)
        self._skip = self._no_grad_slices(model)
        if self.world > 1:
            self.graph.grad_ready_hook = self._on_ready
        self._check_replicas()

    # ------------------------------------------------------------------ data-parallel plumbing
    def _module_slices(self, model) -> Dict[int, Tuple[int, int]]:
        out = {}
        for mod in model.modules():
            names = [n for n, p in mod.named_parameters(prefix=self._prefix(model, mod)) if p.requires_grad]
            if not names:
                continue
            offs = [self.flat.offsets[n] for n in names if n in self.flat.offsets]
            if not offs:
                continue
            a = min(o for o, _ in offs)
            b = max(o + k for o, k in offs)
            out[id(mod)] = (a, b)
        return out

    @staticmethod
    def _prefix(model, mod) -> str:
        for n, m in model.named_modules():
            if m is mod:
                return n
        return ""

    def _no_grad_slices(self, model):
        out = []
        for name in ("point_head", "depth_head"):
            m = getattr(model, name, None)
            if m is not None and id(m) in self._slices:
                out.append(self._slices[id(m)])
        return out

    def _check_replicas(self) -> None:
        """DDP broadcasts rank 0's parameters at construction: do the same."""
        if self.world > 1:
            dist.broadcast(self.flat.data, src=dist.get_global_rank(self.group, 0) if hasattr(dist, "get_global_rank")
                           else 0, group=self.group)
            self.graph.invalidate()

    def _reduce(self, a: int, b: int) -> None:
        if b > a:
            self._works.append(dist.all_reduce(self.flat.grad[a:b], group=self.group, async_op=True))
            self._reduced[a] = (a, b)

    def _on_ready(self, module) -> None:
        if module is not None:
            sl = self._slices.get(id(module))
            if sl is not None and sl[0] not in self._reduced:
                self._reduce(*sl)
            return
        # everything not reduced yet (and not a zero-grad head): the remaining contiguous gaps
        done = sorted(list(self._reduced.values()) + self._skip)
        pos = 0
        for a, b in done:
            if a > pos:
                self._reduce(pos, a)
            pos = max(pos, b)
        if pos < self.flat.numel:
            self._reduce(pos, self.flat.numel)

    # ------------------------------------------------------------------ the step
    def step(self, images: Tensor, no_reloc_list: List[int], reloc_list: List[int], batch: dict,
             fix_rank: int = 300) -> Dict[str, float]:
        # the loss's batch tensors go to the device first, while the stream is idle: a host tensor's
        # copy blocks the host until the stream reaches it, so in the middle of the step it stalled the
        # launch queue behind the whole forward (imc_loss converts the same way; no-ops afterwards)
        dev = images.device
        lb = {k: batch[k].to(device=dev, dtype=torch.int32 if k in ("src_idx", "dst_idx") else torch.float32).contiguous()
              for k in ("K_prime_to_K", "src_idx", "dst_idx", "src_coords", "dst_coords", "src_depth", "dst_depth")}
        self.opt.zero_grad()
        self._works, self._reduced = [], {}
        pose = self.graph.forward(images, no_reloc_list, reloc_list, fix_rank=fix_rank)
        H, W = images.shape[-2], images.shape[-1]
        loss, d_enc = imc_loss(pose[0], (H, W), lb["K_prime_to_K"], bool(batch["shared_focal"]), lb["src_idx"],
                               lb["dst_idx"], lb["src_coords"], lb["dst_coords"], lb["src_depth"],
                               lb["dst_depth"], self.cdf, grad_scale=self.scaler.get_scale())
        self.graph.backward(d_enc[None])
        for w in self._works:
            w.wait()
        self._works = []
        # the bf16 / transposed weight packs are refreshed from the (possibly unchanged, if the update
        # was skipped) fp32 weights before the host reads found_inf back
        found = self.scaler.step(self.opt, world_size=self.world, before_sync=self.graph.refresh_packs)
        self.scaler.update()
        lr = self.sched.step()
        self.steps_done += 1
        return {"loss": float(loss.item()), "lr": lr, "skipped": found}

    def save_checkpoint(self, checkpoint_dir, loss=None) -> Path:
        """Rank 0 saves (train_imc.py:426-428 guards the call with is_main_process)."""
        return save_checkpoint(self.graph.model, self.opt, self.sched, self.scaler, self.steps_done, loss,
                               checkpoint_dir)
