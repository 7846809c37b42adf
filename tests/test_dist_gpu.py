"""Frame-sharded aggregator with the real HIP kernels: 2 or 3 ranks sharing cuda:0 (gloo
collectives on device tensors — the GPU box has one GPU; the driver's 8-GPU run uses
RCCL).  Covers even and uneven anchor / query splits, the overlapped local-then-remote
global attention with its LSE merge (sr_attn_merge; a two-segment remote pass on the middle
rank of 3), and BASELINE config 2 (N=8 views @518) on 2 ranks.  The concatenated per-rank
results must reproduce the reference golden vectors at the full-model bounds (goldens.PARITY_TOL:
fp32 1e-5; bf16 1e-2 features / 2e-3 poses rel-L2), every measured error printed."""

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
from goldens import parity_tol  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir, golden, mode, overlap, backend="gloo", shard=True):
    try:
        _work(rank, world, port, out_dir, golden, mode, overlap, backend, shard)
    except BaseException:  # name the rank that failed first (its peers then only see closed connections)
        import traceback
        print(f"RANK {rank}/{world} FAILED:\n{traceback.format_exc()}", flush=True)
        raise


def _work(rank, world, port, out_dir, golden, mode, overlap, backend, shard):
    for p in (REPO, os.path.join(REPO, "self-supervise-sfm_amd"), HERE):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    if backend == "nccl":
        torch.cuda.set_device(rank)
    dist.init_process_group(backend, rank=rank, world_size=world)
    from goldens import load_npz, rule_state_dict
    from sailrecon_amd.models.aggregator import shard_range
    from sailrecon_amd.utils.pose_enc import pose_encoding_to_extri_intri
    from test_parity_gpu import Hot

    if isinstance(golden, dict):  # no reference golden at this size: the synthetic scene's spec
        g = dict(golden)
        g["sample_rows"] = np.sort(np.random.default_rng(5).choice(g["n_views"] * 1374, 512, replace=False))
    else:
        g = load_npz(golden)
    n = int(g["n_views"])
    full = "img" in g
    torch.manual_seed(0)
    if full:  # BASELINE-shape model, reference-sized images
        img = int(g["img"])
        m = Hot(dict(img_size=518, patch_size=14, embed_dim=1024), dict(dim_in=2048)).eval()
        m.load_state_dict(rule_state_dict("state_dict_keys.json"))
        x = torch.rand(n, 3, img, img, generator=torch.Generator().manual_seed(n))
        images = torch.cat([x, x])[None]
        layers = (4, 11, 17, 23)
    else:
        m = Hot(dict(img_size=56, patch_size=14, embed_dim=384, depth=2, num_heads=6,
                     patch_embed="dinov2_vits14_reg", intermediate_layer_idx=[0, 1]),
                dict(dim_in=768, trunk_depth=2, num_heads=6)).eval()
        m.load_state_dict(rule_state_dict("small_state_dict_keys.json"))
        images = torch.from_numpy(g["images"])
        layers = (0, 1)
    m = m.cuda()
    images = images.cuda()
    if shard:
        m.aggregator.set_frame_sharding(dist.group.WORLD)  # nccl: the seed broadcast as a device tensor
    m.aggregator.shard_overlap = overlap
    if backend == "nccl":  # gather_rows' RCCL all_gather_into_tensor on the K/V row layout
        from sailrecon_amd.models.aggregator import gather_rows
        src = torch.randn(37, 2048, device="cuda", dtype=torch.bfloat16)
        dst = torch.empty(37 * world, 2048, device="cuda", dtype=torch.bfloat16)
        for w in gather_rows(dst, src, [37] * world, dist.group.WORLD, rank):
            w.wait()
        assert torch.equal(dst[rank * 37:(rank + 1) * 37], src)
    m.aggregator.generator.manual_seed(0)
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16, enabled=(mode == "bf16")):
        feats, psi, cam_last = m.aggregator(images, list(range(n)), list(range(n, 2 * n)), fix_rank=int(g["fix_rank"]))
        with torch.autocast("cuda", enabled=False):
            poses = m.camera_head([m.aggregator.last_query_cam_tokens[:, :, None]], cam_last)
            ext, intr = pose_encoding_to_extri_intri(poses[-1], (images.shape[-2], images.shape[-1]))
    torch.cuda.synchronize()
    q0, nq = shard_range(n, world, rank)
    res = {"cam_last": cam_last.cpu().numpy(), "pose": np.stack([p.cpu().numpy() for p in poses]),
           "ext": ext.cpu().numpy(), "intr": intr.cpu().numpy()}
    for layer in layers:
        v = feats[layer][0].float().cpu()  # [nq, P, 2C] of this rank's query frames
        if not full:
            res[f"feat_{layer}"] = v.numpy()
            continue
        P = v.shape[1]
        rows = g["sample_rows"]
        mine = rows[(rows >= q0 * P) & (rows < (q0 + nq) * P)] - q0 * P
        res[f"feat_{layer}_rownorm"] = v.norm(dim=-1).numpy()
        res[f"feat_{layer}_cam"] = v[:, 0].numpy()
        res[f"feat_{layer}_rows"] = v.reshape(-1, v.shape[-1])[torch.from_numpy(mine)].numpy()
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), **res)
    dist.barrier()
    dist.destroy_process_group()


def _spawn(tmp_path, world, golden, mode, overlap=True, backend="gloo", shard=True):
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), golden, mode, overlap, backend, shard),
             nprocs=world, join=True)
    return [np.load(tmp_path / f"rank{r}.npz") for r in range(world)]


def _run(tmp_path, world, golden, mode, overlap=True, backend="gloo"):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from goldens import load_npz, rel_l2
    _spawn(tmp_path, world, golden, mode, overlap, backend)
    g = load_npz(golden)
    rs = [np.load(tmp_path / f"rank{r}.npz") for r in range(world)]
    err = {}
    if "img" in g:
        for layer in (4, 11, 17, 23):
            for key in ("rownorm", "cam", "rows"):
                full = np.concatenate([r[f"feat_{layer}_{key}"] for r in rs], axis=0)
                err[f"feat_{layer}_{key}"] = rel_l2(full, g[f"feat_{layer}_{key}"])
    else:
        for layer in (0, 1):
            full = np.concatenate([r[f"feat_{layer}"] for r in rs], axis=0)
            err[f"feat_{layer}"] = rel_l2(full, g[f"feat_{layer}"][0])
    for i, r in enumerate(rs):
        err[f"rank{i}_cam_token_last_layer"] = rel_l2(r["cam_last"], g["cam_token_last_layer"])
        err[f"rank{i}_pose_enc"] = rel_l2(r["pose"], g["pose_enc"])
        if "extrinsic" in g and "img" in g:
            err[f"rank{i}_extrinsic"] = rel_l2(r["ext"], g["extrinsic"])
            err[f"rank{i}_intrinsic"] = rel_l2(r["intr"], g["intrinsic"])
    print(f"PARITY {golden} {mode} sharded world {world} ({backend}, overlap {overlap}):",
          {k: float(f"{v:.3e}") for k, v in err.items()})
    bad = {k: v for k, v in err.items() if not v < parity_tol(k, mode)}
    assert not bad, bad


@pytest.mark.parametrize("mode", ["fp32", "bf16"])
def test_frame_sharded_rccl_world1(tmp_path, mode):
    """The RCCL ("nccl") process group on the box's one GPU: set_frame_sharding's device-tensor
    seed broadcast (aggregator.py set_frame_sharding), gather_rows' all_gather_into_tensor and the
    sharded forward at world 1 against the reference golden (RCCL refuses two ranks on one
    device, so world 2+ over RCCL is the driver's multi-GPU run)."""
    _run(tmp_path, 1, "g1_small_56.npz", mode, backend="nccl")


def test_frame_sharded_two_ranks_one_gpu(tmp_path):
    _run(tmp_path, 2, "g1_small_56.npz", "fp32")


@pytest.mark.parametrize("mode", ["fp32", "bf16"])
@pytest.mark.parametrize("overlap", [True, False])
def test_frame_sharded_three_ranks_uneven(tmp_path, mode, overlap):
    """5 anchors + 5 queries over 3 ranks: 2 / 2 / 1 frames each; rank 1's remote anchors
    are two key segments (rank 0's and rank 2's)."""
    _run(tmp_path, 3, "g1_small_56_n5.npz", mode, overlap)


@pytest.mark.parametrize("mode", ["fp32", "bf16"])
def test_frame_sharded_eight_ranks(tmp_path, mode):
    """9 anchors + 9 queries over 8 ranks sharing the GPU (2 / 1 / ... / 1 frames each): every
    rank's remote anchors are one or two key segments, gathered from seven peers."""
    _run(tmp_path, 8, "g1_small_56_n9.npz", mode)


@pytest.mark.parametrize("mode", ["fp32", "bf16"])
def test_frame_sharded_c2_518_n8_two_ranks(tmp_path, mode):
    """BASELINE config 2 (N=8 views @518) split over 2 ranks: 4 anchors + 4 queries each; the
    global block's local pass runs on 5,496 keys, the remote pass on the other 5,496."""
    _run(tmp_path, 2, "g9_518_n8.npz", mode)


@pytest.mark.parametrize("world,mode", [(2, "fp32"), (3, "bf16"), (3, "fp32"), (8, "bf16")],
                         ids=["2rk-fp32", "3rk-bf16", "3rk-fp32", "8rk-bf16"])
def test_frame_sharded_c3_518_n32(tmp_path, world, mode):
    """BASELINE config 3 (the headline scene, N=32 views @518) frame-sharded
    over 2 ranks (16 / 16 anchors + queries), 3 ranks (the uneven 11 / 11 / 10 split; the
    middle rank's remote global-attention pass has two key segments) and 8 ranks (the driver's
    8-GPU world: 4 + 4 frames per rank, key-split global passes), every rank's features,
    camera tokens and poses against the reference golden g10 (goldens.PARITY_TOL)."""
    _run(tmp_path, world, "g10_518_n32.npz", mode)


@pytest.mark.parametrize("world", [2, 3])
def test_frame_sharded_n64_matches_one_rank(tmp_path, world):
    """The north-star scaling workload (64 views @518, global L = 87,936) sharded over 2 / 3
    ranks against the same scene on one rank without sharding (no reference golden exists at
    this size: the reference needs hours and 30 GB of dense mask on the CPU).  bf16: the sharded
    run splits the global softmax into local / remote passes merged by LSE and key-split
    partials, so it differs from the one-rank run by bf16 rounding only (measured values printed)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from goldens import rel_l2
    spec = {"n_views": 64, "img": 518, "fix_rank": 300}
    (tmp_path / "one").mkdir()
    one = _spawn(tmp_path / "one", 1, spec, "bf16", shard=False)[0]
    rs = _spawn(tmp_path, world, spec, "bf16")
    errs = {}
    for layer in (4, 11, 17, 23):
        for key in ("rownorm", "cam", "rows"):
            full = np.concatenate([r[f"feat_{layer}_{key}"] for r in rs], axis=0)
            errs[f"{layer}_{key}"] = rel_l2(full, one[f"feat_{layer}_{key}"])
    for i, r in enumerate(rs):
        for k in ("cam_last", "pose", "ext"):
            errs[f"rank{i}_{k}"] = rel_l2(r[k], one[k])
    print(f"N=64 sharded over {world} vs one rank (bf16, rel-L2):", {k: float(f"{v:.2e}") for k, v in errs.items()})
    # about 2x the round-4 / round-5 measurements (features <= 2.2e-3, camera tokens 3e-3, pose
    # encodings 2.0e-4, extrinsics 5.2e-4)
    bound = lambda k: 2e-3 if ("pose" in k or "ext" in k) else 6e-3  # noqa: E731
    bad = {k: (v, bound(k)) for k, v in errs.items() if not v < bound(k)}
    assert not bad, bad

