"""Golden vectors for the two-phase KV-cache relocalisation from the REAL
reference SailRecon (read-only import; build container only):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_kvcache.py

Full-size SailRecon(kv_cache=True), seeded synthetic weights (synth_weights rule), 56x56 images
(4x4 patches: every patch is in the anchor subsample), fp32 on CPU.  Phase 1:
tmp_forward(3 anchors, fix_rank=300) with the aggregator generator re-seeded to 0; phase 2:
reloc(image i, memory_save=False, save_depth=True, ret_img=True) for every i, as
train/demo_imc.py:85-104 does.

  g7_kvcache.npz   per query view i: extrinsic_i, intrinsic_i, depth_map_i, dpt_cnf_i,
                   point_map_i, xyz_cnf_i, cam_tokens_i, unproj_i; images

The reference's cached attention moves its CPU-offloaded cache back with an unconditional
``.cuda()`` (attention.py:92).  This container has no GPU, so for this run ``Tensor.cuda`` is
mapped to the identity: only the device placement changes, not the arithmetic.  The script
also checks that reloc(i) equals the one-pass forward with image i as the query frame.
"""

from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "self-supervise-sfm_amd"))
sys.path.insert(0, "/root/reference")
sys.dont_write_bytecode = True

from sailrecon_amd.utils.synth_weights import synth_state_dict_like  # noqa: E402

from sailrecon.models.sail_recon import SailRecon  # noqa: E402

torch.set_num_threads(8)
torch.Tensor.cuda = lambda self, *a, **k: self  # no GPU here: keep the offloaded cache on the CPU
N, HW = 3, 56


def main():
    torch.manual_seed(0)
    m = SailRecon(kv_cache=True).eval()
    m.load_state_dict(synth_state_dict_like(m))
    images = torch.rand(N, 3, HW, HW, generator=torch.Generator().manual_seed(7))
    out = dict(images=images.numpy())
    with torch.no_grad():
        m.aggregator.generator.manual_seed(0)
        m.tmp_forward(images, fix_rank=300)
        for i in range(N):
            r = m.reloc(images[i:i + 1], fix_rank=300, memory_save=False, save_depth=True, ret_img=True)[0]
            for k in ("extrinsic", "intrinsic", "depth_map", "dpt_cnf", "point_map", "xyz_cnf", "cam_tokens"):
                out[f"{k}_{i}"] = r[k].float().numpy()
            out[f"unproj_{i}"] = np.asarray(r["point_map_by_unprojection"], dtype=np.float64)
        # sanity: reloc(i) equals the one-pass forward with image i as the query frame
        plain = SailRecon(kv_cache=False).eval()
        plain.load_state_dict(synth_state_dict_like(plain))
        plain.aggregator.generator.manual_seed(0)
        r1 = plain(torch.cat([images, images[1:2]])[None], no_reloc_list=list(range(N)), reloc_list=[N],
                   fix_rank=300)[0]
        print("two-phase vs one-pass pose:", float((r1["extrinsic"] - torch.from_numpy(out["extrinsic_1"])).abs().max()))
    np.savez(os.path.join(HERE, "g7_kvcache.npz"), **out)
    print("g7_kvcache.npz", os.path.getsize(os.path.join(HERE, "g7_kvcache.npz")) // 1024, "KiB")


if __name__ == "__main__":
    main()
