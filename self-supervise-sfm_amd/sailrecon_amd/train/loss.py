"""Self-supervised training loss on the HIP path — mirror of compute_loss
(train/train_imc.py:141-246) and CDFLossIndexPytorch (train/losses/cdf_loss.py:19-242).

``CDFLossIndexPytorch`` keeps the reference constructor (min_val, max_val, num_bins, src_indices,
dst_indices, gradient_smooth, num_nodes) and its smoothing taps (cdf_loss.py:62-84); the
histogram / CDF / PDF / lookup run inside sr_imc_loss together with the geometry, and the
gradient the reference's CDFLossTorchWrapper supplies (pdf * weight) is chained down to the pose
encodings in the same call.  ``compute_loss`` returns the reference's {"loss": ...} plus the
gradient with respect to the query views' pose encodings ("d_pose_enc"), which TrainGraph.backward
consumes (the role of ``scaler.scale(loss).backward()``, train_imc.py:404).
"""

from __future__ import annotations

import ctypes
import math
from typing import Optional, Tuple

import torch

from .. import _lib, ops

Tensor = torch.Tensor


class CDFLossIndexPytorch:
    def __init__(self, min_val: float, max_val: float, num_bins: int, src_indices: Tensor, dst_indices: Tensor,
                 gradient_smooth: float = 0.0001, num_nodes: Optional[int] = None):
        self.min_val, self.max_val, self.num_bins = float(min_val), float(max_val), int(num_bins)
        self.gradient_smooth = gradient_smooth
        self.src_indices = torch.as_tensor(src_indices).long()
        self.dst_indices = torch.as_tensor(dst_indices).long()
        if num_nodes is None:
            num_nodes = int(torch.cat([self.src_indices, self.dst_indices]).max()) + 1
        self.num_nodes = num_nodes
        bw = (self.max_val - self.min_val) / self.num_bins
        if gradient_smooth > 0:  # cdf_loss.py:62-84 (same fp32 ops -> same taps)
            r = max(1, int(gradient_smooth / bw))
            idx = torch.arange(2 * r + 1, dtype=torch.float32) - r
            g = torch.exp(-0.5 * (idx / (gradient_smooth / bw)) ** 2)
            self.smooth = g / torch.sum(g)
        else:
            self.smooth = torch.ones(1)
        self._dev = {}

    def to(self, device):
        return self

    def device_tables(self, device):
        key = str(device)
        if key not in self._dev:
            self._dev[key] = dict(smooth=self.smooth.to(device).contiguous(),
                                  src=self.src_indices.int().to(device), dst=self.dst_indices.int().to(device))
        return self._dev[key]


def imc_loss(pose_enc: Tensor, hw: Tuple[int, int], K_prime_to_K: Tensor, shared_focal: bool, src_idx: Tensor,
             dst_idx: Tensor, src_coords: Tensor, dst_coords: Tensor, src_depth: Tensor, dst_depth: Tensor,
             cdf: CDFLossIndexPytorch, grad_scale: float = 1.0, loss_out: Optional[Tensor] = None,
             d_enc_out: Optional[Tensor] = None) -> Tuple[Tensor, Tensor]:
    """(loss [1], d loss / d pose_enc [N, 9] * grad_scale) for pose encodings [N, 9] (device fp32)."""
    dev = pose_enc.device
    enc = pose_enc.reshape(-1, 9).float().contiguous()
    n = enc.shape[0]
    P, K = src_coords.shape[0], src_coords.shape[1]
    f = lambda t: t.to(device=dev, dtype=torch.float32).contiguous()  # noqa: E731
    i = lambda t: t.to(device=dev, dtype=torch.int32).contiguous()  # noqa: E731
    tabs = cdf.device_tables(dev)
    if tabs["src"].numel() == 1 and P > 1:
        raise IndexError("CDFLossIndexPytorch built on single-entry indices cannot index more than one pair "
                         "(cdf_loss.py:147-148)")
    node_src = tabs["src"] if tabs["src"].numel() >= P else None
    node_dst = tabs["dst"] if tabs["dst"].numel() >= P else None
    loss = loss_out if loss_out is not None else torch.empty(1, device=dev, dtype=torch.float32)
    d_enc = d_enc_out if d_enc_out is not None else torch.empty(n, 9, device=dev, dtype=torch.float32)
    L = _lib.load()
    ws_n = L.sr_imc_loss_workspace(n, P, K, cdf.num_nodes, cdf.num_bins)
    ws = ops._train_ws(dev, "imc_loss", ws_n)
    kp, sc, dc, sd, dd = f(K_prime_to_K), f(src_coords), f(dst_coords), f(src_depth), f(dst_depth)
    si, di = i(src_idx), i(dst_idx)
    d = _lib.ImcLossDesc()
    d.enc, d.n_views, d.H, d.W = ops._p(enc), n, int(hw[0]), int(hw[1])
    d.kp2k, d.shared_focal = ops._p(kp), int(bool(shared_focal))
    d.n_pairs, d.n_points = P, K
    d.src_idx, d.dst_idx = ops._p(si), ops._p(di)
    d.src_coords, d.dst_coords, d.src_depth, d.dst_depth = ops._p(sc), ops._p(dc), ops._p(sd), ops._p(dd)
    d.node_src, d.node_dst = ops._p(node_src), ops._p(node_dst)
    d.n_nodes = cdf.num_nodes
    d.min_val, d.max_val, d.num_bins = cdf.min_val, cdf.max_val, cdf.num_bins
    d.smooth_w, d.smooth_radius = ops._p(tabs["smooth"]), tabs["smooth"].numel() // 2
    d.grad_scale = float(grad_scale)
    d.loss, d.d_enc, d.workspace = ops._p(loss), ops._p(d_enc), ops._p(ws)
    _lib.check(L.sr_imc_loss(ops._stream(enc), ctypes.byref(d)), "sr_imc_loss")
    return loss, d_enc


def compute_loss(predictions, batch, device, cdf_loss_module: CDFLossIndexPytorch, do_record: bool = False,
                 image_hw: Tuple[int, int] = (518, 518), grad_scale: float = 1.0) -> dict:
    """train_imc.py:141-246 on the HIP path.  ``predictions``: a list of per-view dicts with
    "pose_enc" ([1, 9] or [9]) like the reference's, or one dict / tensor holding the query
    views' [1, N, 9] pose encoding.  Returns {"loss": [1] tensor, "d_pose_enc": [N, 9]}."""
    if do_record:
        raise NotImplementedError("plot data (get_frame_statistics) is not mirrored")
    if isinstance(predictions, Tensor):
        enc = predictions
    elif isinstance(predictions, dict):
        enc = predictions["pose_enc"]
    else:
        enc = torch.cat([p["pose_enc"].reshape(-1, 9) for p in predictions], 0)
    loss, d_enc = imc_loss(enc.to(device), image_hw, batch["K_prime_to_K"], bool(batch["shared_focal"]),
                           batch["src_idx"], batch["dst_idx"], batch["src_coords"], batch["dst_coords"],
                           batch["src_depth"], batch["dst_depth"], cdf_loss_module, grad_scale=grad_scale)
    return {"loss": loss, "d_pose_enc": d_enc}
