"""Synthetic IMC2021-shaped training batches (the dataset and its HDF5 reader are absent here:
datasets/imc2021.py:260-301 + collate_fn).  A batch holds, like the reference's:
  rgb_processed [N, 3, S, S] in [0, 1], K_prime_to_K [N, 3, 3], shared_focal,
  src_idx / dst_idx [P], src_coords / dst_coords [P, K, 2], src_depth / dst_depth [P, K]
Pairs default to the chain (0,1), (1,2), ...; correspondences are random pixels displaced by a
few pixels with positive depths, so residuals land inside the CDF's [0, 15) log range."""

from __future__ import annotations

from typing import List, Optional, Tuple

import torch


def synthetic_batch(n_views: int, n_points: int = 1024, size: int = 518, seed: int = 0,
                    pairs: Optional[List[Tuple[int, int]]] = None, shared_focal: bool = False) -> dict:
    g = torch.Generator().manual_seed(seed)
    if pairs is None:
        pairs = [(i, i + 1) for i in range(n_views - 1)] or [(0, 0)]
    P = len(pairs)
    s = 0.8 + 0.4 * torch.rand(n_views, generator=g)
    kp = torch.zeros(n_views, 3, 3)
    kp[:, 0, 0] = s
    kp[:, 1, 1] = s
    kp[:, 0, 2] = 20 * torch.randn(n_views, generator=g)
    kp[:, 1, 2] = 20 * torch.randn(n_views, generator=g)
    kp[:, 2, 2] = 1
    src = torch.rand(P, n_points, 2, generator=g) * (size - 20) + 10
    dst = src + 6 * torch.randn(P, n_points, 2, generator=g)
    sd = 1 + 4 * torch.rand(P, n_points, generator=g)
    dd = sd * (1 + 0.05 * torch.randn(P, n_points, generator=g))
    return dict(rgb_processed=torch.rand(n_views, 3, size, size, generator=g), K_prime_to_K=kp,
                shared_focal=shared_focal, src_idx=torch.tensor([a for a, _ in pairs]),
                dst_idx=torch.tensor([b for _, b in pairs]), src_coords=src, dst_coords=dst, src_depth=sd,
                dst_depth=dd)
