"""Golden vectors for the self-supervised training loss from the REAL
reference modules (read-only import; build container only):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_loss.py

Imports the reference's CDFLossIndexPytorch (train/losses/cdf_loss.py:19-242), its projective
geometry (train/utils/geometry.py: backproject_and_reproject[_with_approximation],
compute_relative_pose, compute_projective_residual) and pose decode
(sailrecon/utils/pose_enc.py:68-135), and composes them in the order of compute_loss
(train/train_imc.py:141-246; that file itself imports packages absent here — eval, tensorboard —
so its 40-line body is followed step by step below).  fp32 on CPU, autograd for the gradient of
the loss with respect to the pose encodings (the camera head's output).

Cases (g8_loss.npz, prefix per case):
  dummy   train_epoch's own setup (train_imc.py:334-350): CDF module built on the dummy indices
          [0] / [0] (one histogram), 2 query views, one pair, 700 points
  shared  as dummy with batch['shared_focal'] = True (averaged recovered intrinsics)
  multi   4 views, 3 pairs x 300 points, CDF nodes = the pairs' frame indices (4 histograms)
"""

from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, "/root/reference")
sys.path.insert(0, "/root/reference/train")
sys.dont_write_bytecode = True

from losses.cdf_loss import CDFLossIndexPytorch  # noqa: E402
from utils.geometry import (backproject_and_reproject, backproject_and_reproject_with_approximation,  # noqa: E402
                            compute_projective_residual, compute_relative_pose)

from sailrecon.utils.pose_enc import pose_encoding_to_extri_intri  # noqa: E402

H = W = 518


def make_case(seed, n_views, pairs, npts, shared, nodes):
    g = torch.Generator().manual_seed(seed)
    T = 0.3 * torch.randn(n_views, 3, generator=g)
    q = torch.randn(n_views, 4, generator=g) * 0.2
    q[:, 3] += 1.0
    fov = 0.9 + 0.3 * torch.rand(n_views, 2, generator=g)
    enc = torch.cat([T, q, fov], -1)
    s = 0.5 + torch.rand(n_views, generator=g)
    kp2k = torch.zeros(n_views, 3, 3)
    kp2k[:, 0, 0] = s
    kp2k[:, 1, 1] = s
    kp2k[:, 0, 2] = 40 * torch.randn(n_views, generator=g)
    kp2k[:, 1, 2] = 40 * torch.randn(n_views, generator=g)
    kp2k[:, 2, 2] = 1
    P = len(pairs)
    src_idx = torch.tensor([a for a, _ in pairs])
    dst_idx = torch.tensor([b for _, b in pairs])
    src_coords = torch.rand(P, npts, 2, generator=g) * torch.tensor([W * 0.8, H * 0.8]) + 50
    dst_coords = src_coords + 25 * torch.randn(P, npts, 2, generator=g)
    src_depth = 1 + 4 * torch.rand(P, npts, generator=g)
    dst_depth = src_depth * (1 + 0.1 * torch.randn(P, npts, generator=g))
    return dict(enc=enc, kp2k=kp2k, src_idx=src_idx, dst_idx=dst_idx, src_coords=src_coords, dst_coords=dst_coords,
                src_depth=src_depth, dst_depth=dst_depth, shared=shared, nodes_src=torch.tensor(nodes[0]),
                nodes_dst=torch.tensor(nodes[1]))


def reference_loss(c):
    """compute_loss, train_imc.py:141-246, with predictions from pose_encoding_to_extri_intri."""
    enc = c["enc"].clone().requires_grad_(True)
    extrinsic, intrinsic = pose_encoding_to_extri_intri(enc[None], (H, W))      # sail_recon.py:122-126
    predicted_intrinsics_batched = intrinsic[0]                                     # :157
    recovered = torch.bmm(c["kp2k"], predicted_intrinsics_batched)                 # :166
    if c["shared"]:                                                                 # :169-174
        recovered = recovered.mean(0, keepdim=True).repeat(recovered.shape[0], 1, 1)
    poses = extrinsic[0]                                                            # :177
    src_K, dst_K = recovered[c["src_idx"]], recovered[c["dst_idx"]]                 # :188-191
    rel = compute_relative_pose(poses[c["src_idx"]], poses[c["dst_idx"]])          # :194
    P = c["src_coords"].shape[0]
    ones = torch.ones(P, 1)
    pred, valid = backproject_and_reproject(c["src_coords"], c["src_depth"], src_K, dst_K, rel, ones)   # :202-209
    res = compute_projective_residual(pred, c["dst_coords"]) * valid.float()       # :212-215
    pred2, valid2 = backproject_and_reproject_with_approximation(                   # :219-228
        c["src_coords"], c["src_depth"], c["dst_depth"], src_K, dst_K, rel, ones, ones)
    res2 = compute_projective_residual(pred2, c["dst_coords"]) * valid2.float()    # :231-234
    rl, rl2 = torch.log1p(res), torch.log1p(res2)                                   # :237-238
    w, w2 = valid.float(), valid2.float()
    cdf = CDFLossIndexPytorch(0.0, 15.0, 250, c["nodes_src"], c["nodes_dst"], gradient_smooth=0.05)  # :334-350
    a, b = cdf(rl, w)
    reg = (a.mean() + b.mean()) / 2.0                                               # :246-247
    a2, b2 = cdf(rl2, w2)
    approx = (a2.mean() + b2.mean()) / 2.0
    loss = (reg + approx) / 2.0                                                     # :254
    loss.backward()
    return dict(loss=loss.detach(), grad=enc.grad, rl=rl.detach(), rl2=rl2.detach(), cdf_src=a.detach(),
                cdf_dst=b.detach())


def main():
    torch.manual_seed(0)
    cases = {
        "dummy": make_case(1, 2, [(0, 1)], 700, False, ([0], [0])),
        "shared": make_case(2, 2, [(1, 0)], 700, True, ([0], [0])),
        "multi": make_case(3, 4, [(0, 1), (1, 2), (3, 0)], 300, False, ([0, 1, 3], [1, 2, 0])),
    }
    out = {}
    for name, c in cases.items():
        r = reference_loss(c)
        for k, v in c.items():
            out[f"{name}/{k}"] = np.asarray(v.numpy() if torch.is_tensor(v) else v)
        for k, v in r.items():
            out[f"{name}/out_{k}"] = v.numpy()
        print(name, "loss", float(r["loss"]), "|grad|", float(r["grad"].norm()))
    np.savez_compressed(os.path.join(HERE, "g8_loss.npz"), **out)


if __name__ == "__main__":
    main()
