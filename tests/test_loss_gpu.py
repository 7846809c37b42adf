"""IMC training loss on the HIP path (sr_imc_loss) against the reference modules' goldens
(tests/golden/make_golden_loss.py: CDFLossIndexPytorch + geometry + pose decode composed as
compute_loss, autograd for d loss / d pose encoding).  fp32 per point like the reference;
histogram counts are exact, so bins agree: loss within 1e-5, gradient 1e-4 rel-L2."""

import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("case", ["dummy", "shared", "multi"])
def test_imc_loss_matches_reference(golden_dir, case):
    from sailrecon_amd.train.loss import CDFLossIndexPytorch, imc_loss
    z = np.load(os.path.join(golden_dir, "g8_loss.npz"))
    g = lambda k: torch.from_numpy(z[f"{case}/{k}"])  # noqa: E731
    cdf = CDFLossIndexPytorch(0.0, 15.0, 250, g("nodes_src"), g("nodes_dst"), gradient_smooth=0.05)
    loss, d_enc = imc_loss(g("enc").to(DEV), (518, 518), g("kp2k"), bool(z[f"{case}/shared"]), g("src_idx"),
                           g("dst_idx"), g("src_coords"), g("dst_coords"), g("src_depth"), g("dst_depth"), cdf,
                           grad_scale=4.0)
    ref_l = float(z[f"{case}/out_loss"])
    assert abs(float(loss) - ref_l) <= 1e-5 * abs(ref_l)
    ref = g("out_grad")
    assert float((d_enc.cpu() / 4.0 - ref).norm() / ref.norm()) < 1e-4


def test_imc_loss_dummy_indices_single_pair_only():
    """train_epoch's dummy [0]/[0] module cannot index more than one pair (as the reference)."""
    from sailrecon_amd.train.loss import CDFLossIndexPytorch, imc_loss
    cdf = CDFLossIndexPytorch(0.0, 15.0, 250, torch.tensor([0]), torch.tensor([0]), gradient_smooth=0.05)
    z = torch.zeros(2, 10, 2)
    with pytest.raises(IndexError):
        imc_loss(torch.zeros(2, 9, device=DEV), (518, 518), torch.eye(3).expand(2, 3, 3), False,
                 torch.tensor([0, 1]), torch.tensor([1, 0]), z, z, torch.ones(2, 10), torch.ones(2, 10), cdf)
