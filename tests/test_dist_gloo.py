"""Frame-sharded aggregator on a CPU gloo world of 2 ranks.

Each rank owns half of the anchor frames and half of the query frames; the global
block all-gathers anchor K/V, the global_reloc block all-gathers the anchor-subsample
K/V, and the camera head runs replicated on gathered camera tokens.  The C-ABI
semantics come from tests/cpu_ops.py (no GPU here); on the GPU box the same code
path runs libsfm_amd.so kernels with RCCL collectives.  The gathered result must
equal the reference's golden vectors (and therefore the single-process result).
"""

import os
import socket
import sys

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


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
    torch.set_num_threads(2)
    import cpu_ops
    from goldens import load_npz
    from test_host_cpu import small_model

    g = load_npz("g1_small_56.npz")
    images = torch.from_numpy(g["images"])
    m = small_model()
    m.aggregator.set_frame_sharding(dist.group.WORLD)
    m.aggregator.generator.manual_seed(0)  # identical draws on every rank
    with cpu_ops.installed(), torch.no_grad():
        feats, psi, cam_last = m.aggregator(images, [0, 1], [2, 3], fix_rank=int(g["fix_rank"]))
        poses = m.camera_head([m.aggregator.last_query_cam_tokens[:, :, None]], cam_last)
    # gather every rank's query maps
    res = {}
    for layer in (0, 1):
        loc = feats[layer].contiguous()
        full = [torch.empty_like(loc) for _ in range(world)]
        dist.all_gather(full, loc)
        res[f"feat_{layer}"] = torch.cat(full, dim=1).numpy()
    res["cam_last"] = cam_last.numpy()
    res["pose"] = np.stack([p.numpy() for p in poses])
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), **res)
    dist.barrier()
    dist.destroy_process_group()


def test_frame_sharded_world2_matches_reference(tmp_path):
    from goldens import load_npz, rel_l2
    port = _free_port()
    mp.spawn(_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    g = load_npz("g1_small_56.npz")
    for rank in range(2):
        r = np.load(tmp_path / f"rank{rank}.npz")
        for layer in (0, 1):
            assert rel_l2(r[f"feat_{layer}"], g[f"feat_{layer}"]) < 1e-5
        assert rel_l2(r["cam_last"], g["cam_token_last_layer"]) < 1e-5
        assert rel_l2(r["pose"], g["pose_enc"]) < 1e-5
