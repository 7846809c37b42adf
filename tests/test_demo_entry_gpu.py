"""The demo_imc_forward.py entry flow (tools/demo_imc_forward.py, reference train/demo_imc_forward.py
:25-143) end to end on the HIP path: full SailRecon (all heads) with the seeded weights at 224 px,
N = 2 synthetic views duplicated to 4 frames, bf16 autocast; the per-view predictions equal a
direct SailRecon.forward with the same draws, and the three scene outputs are written."""

import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_demo_imc_forward_flow(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import demo_imc_forward as D
    model = D.load_model(None, "cuda", img_size=224)
    model.aggregator.generator.manual_seed(0)
    res = D.demo(model=model, num_images=2, max_scenes=1, out_dir=str(tmp_path), img_size=224, verbose=False)
    assert len(res) == 1 and len(res[0]) == 2
    keys = {"extrinsic", "intrinsic", "point_map_by_unprojection", "point_map", "rgbs", "xyz_cnf", "depth_map",
            "dpt_cnf", "cam_tokens", "images"}
    for p in res[0]:
        assert set(p) == keys
        assert not p["extrinsic"].is_cuda
    # the same forward called directly (same images, same subsample draws)
    images = D.scene_images(None, 2, 0, 224, "cuda")
    model.aggregator.generator.manual_seed(0)
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        direct = model(torch.cat([images, images]), no_reloc_list=[0, 1], reloc_list=[2, 3], fix_rank=300)
    for a, b in zip(res[0], direct):
        assert torch.equal(a["extrinsic"], b["extrinsic"].cpu())
        assert torch.equal(a["depth_map"], b["depth_map"].cpu())
    out = tmp_path / "scene_000_scene000_"
    poses = np.loadtxt(out / "pred.txt")
    assert poses.shape == (2, 12)
    for i, p in enumerate(res[0]):
        T = np.vstack([p["extrinsic"][0].float().numpy(), [0, 0, 0, 1]])
        assert np.allclose(poses[i].reshape(3, 4), np.linalg.inv(T)[:3], rtol=1e-5, atol=1e-6)
    head = (out / "pred.ply").read_bytes()[:400].split(b"end_header\n")[0].decode()
    nv = int(head.split("element vertex ")[1].split()[0])
    assert 0 < nv <= 2 * 224 * 224
    assert "Number of Predictions: 2" in (out / "scene_info.txt").read_text()
