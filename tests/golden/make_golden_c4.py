"""Golden vectors for BASELINE config 4 — one self-supervised training step's gradients at the
configuration size (16 views @518 -> 32 frames, L_g = 21,984) — from the REAL reference
aggregator + camera head (read-only import; build container only, ~1 h on 8 cores, ~25 GB RSS):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_c4.py            (fp32 -> g12_c4_train.npz)
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_c4.py --bf16     (-> g12_c4_train_bf16.npz)

The model runs in train mode, which makes the reference checkpoint every block itself
(aggregator.py:658-660,722-724,757-759; vision_transformer.py:268) — that is what fits the fp32
autograd graph in memory.  fp32 throughout (no autocast: the golden is the exact reference math).
Weights: the seeded rule (sailrecon_amd/utils/synth_weights.py) on the reference state_dict keys.
Batch: train.data.synthetic_batch(16, n_points=1024, size=518, seed=0) — the kbench/bench C4
batch (15 chained pairs), duplicated into anchors + queries as train_imc.py:107-138 does.
Loss: oracle.sfm_oracle.imc_loss (compute_loss, train_imc.py:141-246 — pinned to the reference's
own CDFLossIndexPytorch / geometry by g8_loss.npz within 1e-6) with per-frame CDF nodes
(CDFLossIndexPytorch(0, 15, 250, src_idx, dst_idx, gradient_smooth=0.05, num_nodes=16)).

--bf16 runs the same reference step under torch.autocast("cpu", dtype=torch.bfloat16) on the
aggregator (train_imc.py:385; the camera head and loss stay fp32, sail_recon.py:118-119): the
reference's OWN bf16-vs-fp32 gradient gap at these positions, which bounds what a bf16 training
path can be asked to match (tests/test_c4_golden_gpu.py).

g12_c4_train.npz holds: the loss; the last camera iteration's pose encodings and d loss / d enc;
the replayed subsample indices; the L2 norm of every parameter's gradient (grad_norm/<name>);
and for ~60 parameters across every stack (DINO, frame, global, global_reloc blocks 0 / 12 / 23,
patch embed, special tokens, camera head) the gradient values at seeded element positions
(grad_idx/<name>, grad_val/<name>; whole tensors up to 8,192 elements).
"""

from __future__ import annotations

import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "self-supervise-sfm_amd"))
sys.path.insert(0, REPO)
sys.path.insert(0, "/root/reference")
sys.dont_write_bytecode = True

from oracle import sfm_oracle as O  # noqa: E402
from sailrecon_amd.train.data import synthetic_batch  # noqa: E402
from sailrecon_amd.utils.synth_weights import synth_state_dict_like  # noqa: E402

from sailrecon.heads.camera_head import CameraHead  # noqa: E402
from sailrecon.models.aggregator import Aggregator  # noqa: E402

torch.set_num_threads(8)
N_VIEWS, IMG, FIX_RANK = 16, 518, 300
SAMPLE = 4096


class Hot(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.aggregator = Aggregator(img_size=518, patch_size=14, embed_dim=1024)
        self.camera_head = CameraHead(dim_in=2048)


def sampled_params(names):
    out = ["aggregator.patch_embed.patch_embed.proj.weight", "aggregator.patch_embed.patch_embed.proj.bias",
           "aggregator.patch_embed.cls_token", "aggregator.patch_embed.pos_embed",
           "aggregator.patch_embed.register_tokens", "aggregator.patch_embed.norm.weight",
           "aggregator.camera_token", "aggregator.register_token", "aggregator.camera_token_reloc",
           "aggregator.register_token_reloc",
           "camera_head.token_norm.weight", "camera_head.embed_pose.weight", "camera_head.poseLN_modulation.1.weight",
           "camera_head.trunk.0.attn.qkv.weight", "camera_head.trunk.3.mlp.fc2.weight",
           "camera_head.trunk_norm.weight", "camera_head.pose_branch.fc1.weight", "camera_head.pose_branch.fc2.weight"]
    for stack in ("patch_embed.blocks", "frame_blocks", "global_blocks", "global_reloc_blocks"):
        for i in (0, 12, 23):
            p = f"aggregator.{stack}.{i}."
            out += [p + s for s in ("attn.qkv.weight", "attn.qkv.bias", "attn.proj.weight", "mlp.fc1.weight",
                                    "mlp.fc2.bias", "norm1.weight", "ls1.gamma", "ls2.gamma")]
            if stack != "patch_embed.blocks":
                out.append(p + "attn.k_norm.weight")
    missing = [n for n in out if n not in names]
    assert not missing, missing
    return out


def main():
    bf16 = "--bf16" in sys.argv[1:]
    t0 = time.time()
    torch.manual_seed(0)
    m = Hot().train()
    sd = synth_state_dict_like(m)
    m.load_state_dict(sd)
    del sd
    b = synthetic_batch(N_VIEWS, n_points=1024, size=IMG, seed=0)
    images = torch.cat([b["rgb_processed"], b["rgb_processed"]])[None]  # train_imc.py:107-138
    na, nq = list(range(N_VIEWS)), list(range(N_VIEWS, 2 * N_VIEWS))
    m.aggregator.generator.manual_seed(0)
    print(f"built in {time.time() - t0:.1f}s", flush=True)
    t1 = time.time()
    with torch.autocast("cpu", dtype=torch.bfloat16, enabled=bf16):
        feats, psi, cam_last = m.aggregator(images, na, nq, fix_rank=FIX_RANK)
    feats = {k: v.float() for k, v in feats.items()}  # output_dict: layer -> [B, S, P, 2C]
    poses = m.camera_head(feats, cam_last.float())
    enc = poses[-1][0]
    enc.retain_grad()
    print(f"forward {time.time() - t1:.1f}s", flush=True)
    loss = O.imc_loss(enc, (IMG, IMG), b["K_prime_to_K"], bool(b["shared_focal"]), b["src_idx"], b["dst_idx"],
                      b["src_coords"], b["dst_coords"], b["src_depth"], b["dst_depth"], b["src_idx"], b["dst_idx"],
                      N_VIEWS, 0.0, 15.0, 250, 0.05)
    t2 = time.time()
    loss.backward()
    print(f"backward {time.time() - t2:.1f}s, loss {float(loss):.6f}", flush=True)
    n_patch = (IMG // 14) ** 2
    gsub = torch.Generator().manual_seed(0)
    sub = np.zeros((24, N_VIEWS, FIX_RANK), dtype=np.int64)
    for l in range(24):
        for a in range(N_VIEWS):
            sub[l, a] = torch.randperm(n_patch, generator=gsub)[:FIX_RANK].numpy()
    out = dict(loss=np.float64(loss.item()), pose_enc=enc.detach().numpy(), d_enc=enc.grad.numpy(), sub_idx=sub,
               n_views=np.int64(N_VIEWS), img=np.int64(IMG), fix_rank=np.int64(FIX_RANK),
               ref_step_s=np.float64(time.time() - t1))
    params = dict(m.named_parameters())
    for n, p in params.items():
        out[f"grad_norm/{n}"] = np.float64(0.0 if p.grad is None else p.grad.double().norm().item())
    rng = np.random.default_rng(0)
    for n in sampled_params(params):
        g = params[n].grad.reshape(-1)
        idx = np.arange(g.numel()) if g.numel() <= 2 * SAMPLE else np.sort(rng.choice(g.numel(), SAMPLE,
                                                                                        replace=False))
        out[f"grad_idx/{n}"] = idx.astype(np.int64)
        out[f"grad_val/{n}"] = g[torch.from_numpy(idx)].numpy().astype(np.float32)
    fname = "g12_c4_train_bf16.npz" if bf16 else "g12_c4_train.npz"
    np.savez_compressed(os.path.join(HERE, fname), **out)
    print(f"wrote {fname} ({os.path.getsize(os.path.join(HERE, fname)) // 1024} KiB) in {time.time() - t0:.1f}s",
          flush=True)


if __name__ == "__main__":
    main()
