"""Data-parallel gradient reduction of the training step (train/step.py, the role of DDP's
buckets, train_imc.py:474) on CPU: 2 gloo ranks, per-module slices reduced as the backward
would report them ready, then the remaining gaps; every gradient ends up summed over ranks,
the zero-grad DPT heads are skipped, and rank 0's parameters are broadcast at construction."""

import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    for p in (REPO, os.path.join(REPO, "self-supervise-sfm_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from sailrecon_amd.heads.camera_head import CameraHead
        from sailrecon_amd.heads.dpt_head import DPTHead
        from sailrecon_amd.models.aggregator import Aggregator
        from sailrecon_amd.train.step import Trainer

        class Small(torch.nn.Module):
            def __init__(self):
                super().__init__()
                self.aggregator = Aggregator(img_size=28, patch_size=14, embed_dim=64, depth=2, num_heads=1,
                                             patch_embed="conv", intermediate_layer_idx=[0, 1])
                self.camera_head = CameraHead(dim_in=128, trunk_depth=1, num_heads=1)
                self.depth_head = DPTHead(dim_in=128, output_dim=2, features=16, out_channels=[8, 16, 32, 32],
                                          intermediate_layer_idx=[0, 1, 0, 1])
        torch.manual_seed(100 + rank)  # different init per rank: the broadcast must unify them
        m = Small()
        tr = Trainer(m, group=dist.group.WORLD)
        g = tr.flat.grad
        g.copy_(torch.arange(g.numel(), dtype=torch.float32) * (rank + 1))
        dh = tr._slices[id(m.depth_head)]
        g[dh[0]:dh[1]] = 0.0
        tr._works, tr._reduced = [], {}
        tr._on_ready(m.camera_head)
        tr._on_ready(m.aggregator.global_reloc_blocks[1])
        tr._on_ready(m.aggregator.frame_blocks[0])
        tr._on_ready(None)
        for w in tr._works:
            w.wait()
        expect = torch.arange(g.numel(), dtype=torch.float32) * 3
        expect[dh[0]:dh[1]] = 0.0
        data = [torch.empty_like(tr.flat.data) for _ in range(world)]
        dist.all_gather(data, tr.flat.data)
        q.put((rank, bool(torch.equal(g, expect)), bool(torch.equal(data[0], data[1]))))
    finally:
        dist.destroy_process_group()


def test_grad_allreduce_buckets_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, grads_ok, same in res:
        assert grads_ok, f"rank {rank}: gradients not summed over ranks"
        assert same, f"rank {rank}: replicas differ after the construction broadcast"
