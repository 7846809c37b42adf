"""Frame-sharded aggregator on CPU gloo worlds of 2 and 3 ranks.

Each rank owns a balanced contiguous slice of the anchor frames and of the query frames
(``shard_range``: even and UNEVEN splits); the global block gathers anchor K/V (attending
to the local anchors first and merging the remote pass by LSE, or — overlap off — one
pass after the gather), the global_reloc block gathers the anchor-subsample K/V, and the
camera head runs replicated on gathered camera tokens.  The C-ABI semantics come from
tests/cpu_ops.py (no GPU here); on the GPU box the same code path runs libsfm_amd.so
kernels with RCCL collectives.  The concatenated per-rank results must equal the
reference's golden vectors (and therefore the single-process result).
"""

import os
import socket
import sys

import numpy as np
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


def _lists(g):
    if "no_reloc" in g:
        return [int(i) for i in g["no_reloc"]], [int(i) for i in g["reloc"]]
    n = int(g["n_views"])
    return list(range(n)), list(range(n, 2 * n))


def _worker(rank, world, port, out_dir, golden, overlap):
    for p in (REPO, os.path.join(REPO, "self-supervise-sfm_amd"), HERE):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(2)
    import cpu_ops
    from goldens import load_npz
    from test_host_cpu import small_model

    g = load_npz(golden)
    images = torch.from_numpy(g["images"])
    no_reloc, reloc = _lists(g)
    m = small_model()
    m.aggregator.set_frame_sharding(dist.group.WORLD)
    m.aggregator.shard_overlap = overlap
    m.aggregator.generator.manual_seed(0)  # identical draws on every rank
    with cpu_ops.installed(), torch.no_grad():
        feats, psi, cam_last = m.aggregator(images, no_reloc, reloc, fix_rank=int(g["fix_rank"]))
        poses = m.camera_head([m.aggregator.last_query_cam_tokens[:, :, None]], cam_last)
    res = {f"feat_{layer}": feats[layer].numpy() for layer in (0, 1)}
    res["cam_last"] = cam_last.numpy()
    res["pose"] = np.stack([p.numpy() for p in poses])
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), **res)
    dist.barrier()
    dist.destroy_process_group()


CASES = [  # (world, golden, overlap): anchors / queries per rank
    (2, "g1_small_56.npz", True),       # 1,1
    (2, "g1_small_70.npz", True),       # 2,1  uneven
    (2, "g1_small_70.npz", False),      # 2,1  uneven, one pass after the gather
    (3, "g1_small_70.npz", True),       # 1,1,1
    (3, "g1_small_56_n5.npz", True),    # 2,2,1  uneven
    (3, "g1_small_56_n5.npz", False),
    (3, "g11_small_interleaved.npz", True),  # 1,1,1, permuted + interleaved frame lists
]


@pytest.mark.parametrize("world,golden,overlap", CASES)
def test_frame_sharded_matches_reference(tmp_path, world, golden, overlap):
    from goldens import load_npz, rel_l2
    port = _free_port()
    mp.spawn(_worker, args=(world, port, str(tmp_path), golden, overlap), nprocs=world, join=True)
    g = load_npz(golden)
    rs = [np.load(tmp_path / f"rank{rank}.npz") for rank in range(world)]
    nq = len(_lists(g)[1])
    from sailrecon_amd.models.aggregator import shard_range
    assert [r["feat_0"].shape[1] for r in rs] == [shard_range(nq, world, j)[1] for j in range(world)]
    for layer in (0, 1):
        full = np.concatenate([r[f"feat_{layer}"] for r in rs], axis=1)
        assert rel_l2(full, g[f"feat_{layer}"]) < 1e-5
    for r in rs:
        assert rel_l2(r["cam_last"], g["cam_token_last_layer"]) < 1e-5
        assert rel_l2(r["pose"], g["pose_enc"]) < 1e-5


def test_shard_range_partitions():
    from sailrecon_amd.models.aggregator import shard_range
    for n in range(0, 40):
        for G in range(1, 9):
            parts = [shard_range(n, G, r) for r in range(G)]
            assert sum(c for _, c in parts) == n
            assert max(c for _, c in parts) - min(c for _, c in parts) <= 1
            start = 0
            for s, c in parts:  # contiguous, in rank order
                assert s == start
                start += c
