"""End-to-end parity of the HIP path against the reference's golden vectors.

fp32 parity mode (no autocast): exact-fp32 MFMA GEMMs + fp32 attention.
bf16 mode (under torch.autocast, the demo_imc_forward.py:93 convention): bf16 MFMA
GEMMs / attention with fp32 residual and fp32 camera head (the reference's own bf16-vs-fp32 gap
is 0.7-0.9 %).
Bounds per quantity class (goldens.PARITY_TOL, rel-L2): fp32 1e-5 on features and poses (north
star: pose within 1e-4); bf16 1e-2 on feature maps / camera tokens and 2e-3 on pose encodings /
extrinsics / intrinsics -- about 2x the worst errors measured on MI355X (4.7e-3 / 8.1e-4), under
SURVEY §8(c)'s 2e-2.  Every test prints its measured errors ("PARITY ..." lines).
"""

import numpy as np
import pytest
import torch
import torch.nn as nn

from goldens import load_npz, parity_tol, rel_l2, rule_state_dict

pytestmark = pytest.mark.gpu

DEV = "cuda"


class Hot(nn.Module):
    def __init__(self, agg_kw, cam_kw):
        super().__init__()
        from sailrecon_amd.heads.camera_head import CameraHead
        from sailrecon_amd.models.aggregator import Aggregator
        self.aggregator = Aggregator(**agg_kw)
        self.camera_head = CameraHead(**cam_kw)


def run(model, images, n, fix_rank, mode, lists=None):
    from sailrecon_amd.utils.pose_enc import pose_encoding_to_extri_intri
    S = images.shape[1]
    no_reloc, reloc = lists if lists is not None else (list(range(n)), list(range(n, S)))
    model.aggregator.generator.manual_seed(0)
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16, enabled=(mode == "bf16")):
        feats, psi, cam_last = model.aggregator(images, no_reloc, reloc, fix_rank=fix_rank)
        with torch.autocast("cuda", enabled=False):
            poses = model.camera_head(feats, cam_last)
            ext, intr = pose_encoding_to_extri_intri(poses[-1], (images.shape[-2], images.shape[-1]))
    torch.cuda.synchronize()
    return feats, psi, cam_last, poses, ext, intr


@pytest.fixture(scope="module")
def small_model():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.manual_seed(0)
    m = Hot(dict(img_size=56, patch_size=14, embed_dim=384, depth=2, num_heads=6,
                 patch_embed="dinov2_vits14_reg", intermediate_layer_idx=[0, 1]),
            dict(dim_in=768, trunk_depth=2, num_heads=6)).eval()
    m.load_state_dict(rule_state_dict("small_state_dict_keys.json"))
    return m.to(DEV)


@pytest.mark.parametrize("mode", ["fp32", "bf16"])
@pytest.mark.parametrize("tag", ["56", "70"])
def test_small_end_to_end(small_model, tag, mode):
    g = load_npz(f"g1_small_{tag}.npz")
    n = int(g["n_views"])
    images = torch.from_numpy(g["images"]).to(DEV)
    feats, psi, cam_last, poses, ext, intr = run(small_model, images, n, int(g["fix_rank"]), mode)
    assert psi == 5
    assert np.array_equal(small_model.aggregator.last_subsample_indices[:, 0].numpy(), g["sub_idx"])
    assert feats[-1] is feats[1]
    err = {f"feat_{layer}": rel_l2(feats[layer].cpu().numpy(), g[f"feat_{layer}"]) for layer in (0, 1)}
    err["cam_token_last_layer"] = rel_l2(cam_last.cpu().numpy(), g["cam_token_last_layer"])
    err["pose_enc"] = rel_l2(np.stack([p.cpu().numpy() for p in poses]), g["pose_enc"])
    err["extrinsic"] = rel_l2(ext.cpu().numpy(), g["extrinsic"])
    err["intrinsic"] = rel_l2(intr.cpu().numpy(), g["intrinsic"])
    _assert_tol(err, mode, f"g1_small_{tag}")


@pytest.mark.parametrize("mode", ["fp32", "bf16"])
def test_small_interleaved_lists(small_model, mode):
    """Frame-order semantics (aggregator.py:287-299,351-399): anchors [3, 1, 4] and queries
    [0, 5, 2] interleaved and permuted, frame 0 a query (no anchor takes camera_token[:, 0]);
    outputs in reloc_list / no_reloc_list order, subsample draws in no_reloc_list order."""
    g = load_npz("g11_small_interleaved.npz")
    no_reloc, reloc = g["no_reloc"].tolist(), g["reloc"].tolist()
    images = torch.from_numpy(g["images"]).to(DEV)
    feats, psi, cam_last, poses, ext, intr = run(small_model, images, len(no_reloc), int(g["fix_rank"]), mode,
                                                 lists=(no_reloc, reloc))
    assert np.array_equal(small_model.aggregator.last_subsample_indices[:, 0].numpy(), g["sub_idx"])
    err = {f"feat_{layer}": rel_l2(feats[layer].cpu().numpy(), g[f"feat_{layer}"]) for layer in (0, 1)}
    err["cam_token_last_layer"] = rel_l2(cam_last.cpu().numpy(), g["cam_token_last_layer"])
    err["pose_enc"] = rel_l2(np.stack([p.cpu().numpy() for p in poses]), g["pose_enc"])
    err["extrinsic"] = rel_l2(ext.cpu().numpy(), g["extrinsic"])
    _assert_tol(err, mode, "g11_small_interleaved")


@pytest.mark.parametrize("fused", [False, True], ids=["resid-epilogue", "fused-resid-ln"])
def test_block_kats_fp32(fused, monkeypatch):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from sailrecon_amd.layers.block import Block
    from sailrecon_amd.layers.rope import RotaryPositionEmbedding2D
    from sailrecon_amd import runtime
    from functools import partial
    # fused: the projection's bias epilogue + sr_residual_layernorm (SR_FUSED_RESID_LN=1)
    monkeypatch.setattr(runtime, "_FUSED_RESID_LN", fused)
    g = load_npz("g2_blocks.npz")
    blk = Block(dim=1024, num_heads=16, init_values=0.01, qk_norm=True, rope=RotaryPositionEmbedding2D(100))
    blk.load_state_dict(rule_state_dict("block_state_dict_keys.json", "agg"))
    blk = blk.to(DEV)
    y = blk(torch.from_numpy(g["agg_x"]).to(DEV), pos=torch.from_numpy(g["agg_pos"]).to(DEV))
    assert rel_l2(y.cpu().numpy(), g["agg_y"]) < 1e-5
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = blk(torch.from_numpy(g["agg_x"]).to(DEV), pos=torch.from_numpy(g["agg_pos"]).to(DEV))
    assert rel_l2(y.float().cpu().numpy(), g["agg_y"]) < 2e-2
    blk = Block(dim=1024, num_heads=16, init_values=1.0, norm_layer=partial(nn.LayerNorm, eps=1e-6))
    blk.load_state_dict(rule_state_dict("block_state_dict_keys.json", "dino"))
    y = blk.to(DEV)(torch.from_numpy(g["dino_x"]).to(DEV))
    assert rel_l2(y.cpu().numpy(), g["dino_y"]) < 1e-5
    blk = Block(dim=2048, num_heads=16, init_values=0.01)
    blk.load_state_dict(rule_state_dict("block_state_dict_keys.json", "cam"))
    y = blk.to(DEV)(torch.from_numpy(g["cam_x"]).to(DEV), None, torch.from_numpy(g["cam_mask"]).to(DEV))
    assert rel_l2(y.cpu().numpy(), g["cam_y"]) < 1e-5


@pytest.fixture(scope="module")
def full_model():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.manual_seed(0)
    m = Hot(dict(img_size=518, patch_size=14, embed_dim=1024), dict(dim_in=2048)).eval()
    m.load_state_dict(rule_state_dict("state_dict_keys.json"))
    return m.to(DEV)


def _full_errors(model, fname, mode):
    """rel-L2 of every checked quantity of a full-size golden (feature maps per layer: row norms,
    camera columns, sampled rows; camera tokens; pose encodings; extrinsic / intrinsic)."""
    g = load_npz(fname)
    n, img = int(g["n_views"]), int(g["img"])
    gen = torch.Generator().manual_seed(n)
    x = torch.rand(n, 3, img, img, generator=gen)
    images = torch.cat([x, x])[None].to(DEV)
    feats, psi, cam_last, poses, ext, intr = run(model, images, n, 300, mode)
    assert np.array_equal(model.aggregator.last_subsample_indices[:, 0].numpy(), g["sub_idx"])
    rows = torch.from_numpy(g["sample_rows"])
    err = {}
    for layer in (4, 11, 17, 23):
        v = feats[layer][0].cpu()
        err[f"feat_{layer}_rownorm"] = rel_l2(v.norm(dim=-1).numpy(), g[f"feat_{layer}_rownorm"])
        err[f"feat_{layer}_cam"] = rel_l2(v[:, 0].numpy(), g[f"feat_{layer}_cam"])
        err[f"feat_{layer}_rows"] = rel_l2(v.reshape(-1, v.shape[-1])[rows].numpy(), g[f"feat_{layer}_rows"])
    err["cam_token_last_layer"] = rel_l2(cam_last.cpu().numpy(), g["cam_token_last_layer"])
    err["pose_enc"] = rel_l2(np.stack([p.cpu().numpy() for p in poses]), g["pose_enc"])
    err["extrinsic"] = rel_l2(ext.cpu().numpy(), g["extrinsic"])
    err["intrinsic"] = rel_l2(intr.cpu().numpy(), g["intrinsic"])
    return err


def _assert_tol(err, mode, what):
    """Print every measured error (GPUTEST logs show drift) and check each against its bound."""
    print(f"PARITY {what} {mode}:", {k: float(f"{v:.3e}") for k, v in err.items()})
    bad = {k: (v, parity_tol(k, mode)) for k, v in err.items() if not v < parity_tol(k, mode)}
    assert not bad, bad


def _check_full(model, fname, mode, what=""):
    _assert_tol(_full_errors(model, fname, mode), mode, fname + what)


@pytest.mark.parametrize("mode", ["fp32", "bf16"])
def test_full_c1_224(full_model, mode):
    _check_full(full_model, "g4_c1_224.npz", mode)


@pytest.mark.parametrize("mode", ["fp32", "bf16"])
def test_full_518_n1(full_model, mode):
    _check_full(full_model, "g5_518_n1.npz", mode)


@pytest.mark.parametrize("mode", ["fp32", "bf16"])
def test_full_c2_518_n8(full_model, mode):
    """BASELINE config 2: N=8 views @518 (S=16 frames, L_g = 10,992, L_r = 13,432)."""
    _check_full(full_model, "g9_518_n8.npz", mode)


@pytest.mark.parametrize("mode", ["fp32", "bf16"])
def test_full_c3_518_n32(full_model, mode):
    """BASELINE config 3, the headline workload: N=32 views @518 (S=64 frames, L_g = 43,968)."""
    _check_full(full_model, "g10_518_n32.npz", mode)


@pytest.mark.parametrize("fname", ["g9_518_n8.npz", "g10_518_n32.npz"], ids=["C2", "C3"])
@pytest.mark.parametrize("mode", ["fp32", "bf16"])
def test_full_deferred_residuals(full_model, fname, mode, monkeypatch):
    """proj / fc2 in the plain bias epilogue (their output in the compute dtype,
    as the reference's autocast Linear returns it) with the residual updates folded into the next
    LayerNorm (runtime: SR_FUSED_RESID_LN + SR_DEFER_RESID) -- against the reference goldens at
    the BASELINE workloads."""
    from sailrecon_amd import runtime
    monkeypatch.setattr(runtime, "_FUSED_RESID_LN", True)
    monkeypatch.setattr(runtime, "_DEFER_RESID", True)
    _check_full(full_model, fname, mode, " deferred residuals")


# fp8 global attention (BASELINE C5's precision, opt-in: Aggregator.set_fp8_global) at the C3
# headline scene against the reference's fp32 golden.  No reference output pins an fp8 contract
# (the reference runs bf16 SDPA); the tolerances below are the measured errors with ~2-4x headroom,
# next to bf16's 1e-2 / 2e-3.  Measured on MI355X (round 3, printed by the test): qk feature maps / camera
# tokens <= 4.4e-3, pose encoding / extrinsic / intrinsic <= 6.3e-4; qkv 4.6e-3 / 6.9e-4 -- the fp8
# global attention adds little to the bf16 path's own gap at this scene.
FP8_TOL = {"qk": {"feat": 1e-2, "pose": 3e-3}, "qkv": {"feat": 1e-2, "pose": 3e-3}}


@pytest.mark.parametrize("fp8", ["qk", "qkv"])
def test_full_c3_518_n32_fp8_global(full_model, fp8):
    full_model.aggregator.set_fp8_global(True, fp8_v=(fp8 == "qkv"))
    try:
        err = _full_errors(full_model, "g10_518_n32.npz", "bf16")
    finally:
        full_model.aggregator.set_fp8_global(False)
    print(f"C3 fp8 global ({fp8}) rel-L2 vs the reference fp32 golden:",
          {k: float(f"{v:.3e}") for k, v in err.items()})
    feat = max(v for k, v in err.items() if k.startswith("feat_") or k == "cam_token_last_layer")
    pose = max(err["pose_enc"], err["extrinsic"], err["intrinsic"])
    assert feat < FP8_TOL[fp8]["feat"], err
    assert pose < FP8_TOL[fp8]["pose"], err
