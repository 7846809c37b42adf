"""Training step (train_imc.py:366-411) on the HIP path: Trainer.step =
forward + IMC loss + backward + GradScaler + Adam + cosine-warmup LR, and its data-parallel form
(2 ranks sharing the one GPU of the box, gloo collectives on device tensors; the driver's
multi-GPU node uses RCCL)."""

import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
DEV = "cuda"


def _small():
    from sailrecon_amd.heads.camera_head import CameraHead
    from sailrecon_amd.models.aggregator import Aggregator
    from sailrecon_amd.utils.synth_weights import synth_state_dict_like

    class Hot(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.aggregator = Aggregator(img_size=56, patch_size=14, embed_dim=384, depth=2, num_heads=6,
                                         patch_embed="dinov2_vits14_reg", intermediate_layer_idx=[0, 1])
            self.camera_head = CameraHead(dim_in=768, trunk_depth=2, num_heads=6)
    torch.manual_seed(0)
    m = Hot()
    m.load_state_dict(synth_state_dict_like(m))
    return m


def _batch(seed):
    from sailrecon_amd.train.data import synthetic_batch
    return synthetic_batch(2, n_points=300, size=56, seed=seed)


def test_trainer_step_matches_torch_adam():
    from sailrecon_amd.train.step import Trainer, prepare_model_input
    m = _small().to(DEV)
    tr = Trainer(m, max_lr=2e-4, warmup_steps=10, max_steps=100)
    b = _batch(3)
    imgs, na, nq = prepare_model_input(b["rgb_processed"].to(DEV))
    p0 = tr.flat.data.clone()
    m.aggregator.generator.manual_seed(0)
    out = tr.step(imgs, na, nq, b, fix_rank=10)
    assert np.isfinite(out["loss"]) and not out["skipped"]
    g = tr.flat.grad / tr.scaler.get_scale()
    assert float(g.norm()) > 0
    ref = p0.clone().requires_grad_(True)
    opt = torch.optim.Adam([ref], lr=2e-4, betas=(0.9, 0.999), eps=1e-8)
    ref.grad = g
    opt.step()
    assert float((tr.flat.data - ref.detach()).norm() / (ref.detach() - p0).norm()) < 1e-4
    assert out["lr"] == pytest.approx(2e-4 * 1 / 10)
    # the next forward sees the updated weights (bf16 packs recast in place)
    m.aggregator.generator.manual_seed(0)
    out2 = tr.step(imgs, na, nq, b, fix_rank=10)
    assert np.isfinite(out2["loss"])


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir):
    for p in (REPO, os.path.join(REPO, "self-supervise-sfm_amd"), HERE):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from sailrecon_amd.train.step import Trainer, prepare_model_input
    from test_train_step_gpu import _batch, _small
    m = _small().cuda()
    tr = Trainer(m, max_lr=2e-4, warmup_steps=10, max_steps=100, group=dist.group.WORLD)
    b = _batch(10 + rank)
    imgs, na, nq = prepare_model_input(b["rgb_processed"].cuda())
    m.aggregator.generator.manual_seed(0)
    tr.step(imgs, na, nq, b, fix_rank=10)
    torch.cuda.synchronize()
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), grad=tr.flat.grad.cpu().numpy(),
             data=tr.flat.data.cpu().numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_data_parallel_two_ranks(tmp_path):
    """All-reduced grads = sum of the per-scene grads of a single process; replicas stay equal."""
    from sailrecon_amd.train.loss import CDFLossIndexPytorch, imc_loss
    from sailrecon_amd.train.model import TrainGraph
    from sailrecon_amd.train.step import prepare_model_input
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    r0, r1 = np.load(tmp_path / "rank0.npz"), np.load(tmp_path / "rank1.npz")
    assert np.array_equal(r0["data"], r1["data"])
    m = _small().to(DEV)
    tg = TrainGraph(m)
    cdf = CDFLossIndexPytorch(0.0, 15.0, 250, torch.tensor([0]), torch.tensor([0]), gradient_smooth=0.05)
    tg.flat.zero_grad()
    for rank in (0, 1):
        b = _batch(10 + rank)
        imgs, na, nq = prepare_model_input(b["rgb_processed"].to(DEV))
        m.aggregator.generator.manual_seed(0)
        pose = tg.forward(imgs, na, nq, fix_rank=10)
        _, d = imc_loss(pose[0], (56, 56), b["K_prime_to_K"], False, b["src_idx"], b["dst_idx"], b["src_coords"],
                        b["dst_coords"], b["src_depth"], b["dst_depth"], cdf, grad_scale=2.0 ** 16)
        tg.backward(d[None])
    ref = tg.flat.grad.cpu().numpy()
    assert np.linalg.norm(r0["grad"] - ref) <= 1e-5 * np.linalg.norm(ref)
