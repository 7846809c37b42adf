"""DPT point / depth heads and depth unprojection on the HIP path against
the reference's golden vectors (tests/golden/make_golden_dpt.py) and the CPU oracle.
fp32 end to end (the reference runs its heads with autocast off): tolerance 1e-4 rel-L2."""

import numpy as np
import pytest
import torch

from goldens import DPT_HEADS, DPT_SMALL, dpt_224_inputs, dpt_small_model_sd, load_npz, rel_l2

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL = 1e-4


@pytest.mark.parametrize("kind", ["point", "depth"])
def test_dpt_small_matches_reference(kind):
    g = load_npz("g6_dpt_small.npz")
    m, sd = dpt_small_model_sd(kind)
    m.load_state_dict(sd)
    m = m.to(DEV)
    toks = {l: torch.from_numpy(g[f"tok_{l}"]).to(DEV) for l in DPT_SMALL["intermediate_layer_idx"]}
    preds, conf = m(toks, images=torch.from_numpy(g["images"]).to(DEV), patch_start_idx=5, frames_chunk_size=2)
    assert preds.shape == g[f"{kind}_preds"].shape and conf.shape == g[f"{kind}_conf"].shape
    assert rel_l2(preds.cpu().numpy(), g[f"{kind}_preds"]) < TOL
    assert rel_l2(conf.cpu().numpy(), g[f"{kind}_conf"]) < TOL


def test_dpt_feature_only_matches_reference():
    """DPTHead(feature_only=True) (dpt_head.py:123-126,286-287): the fused, upsampled,
    position-embedded feature map [B, S, features, H, W] against the reference's output."""
    from goldens import dpt_feat_model_sd
    g = load_npz("g6_dpt_feat_small.npz")
    m, sd = dpt_feat_model_sd()
    m.load_state_dict(sd)
    m = m.to(DEV)
    toks = {l: torch.from_numpy(g[f"tok_{l}"]).to(DEV) for l in DPT_SMALL["intermediate_layer_idx"]}
    feat = m(toks, images=torch.from_numpy(g["images"]).to(DEV), patch_start_idx=5, frames_chunk_size=2)
    assert tuple(feat.shape) == g["feat"].shape
    assert rel_l2(feat.cpu().numpy(), g["feat"]) < TOL


def test_dpt_224_matches_reference():
    from sailrecon_amd.heads.dpt_head import DPTHead
    from sailrecon_amd.utils.synth_weights import synth_state_dict_like
    g = load_npz("g6_dpt_224.npz")
    toks, images = dpt_224_inputs()
    toks = {l: t.to(DEV) for l, t in toks.items()}
    images = images.to(DEV)
    for kind in ("point", "depth"):
        m = DPTHead(dim_in=2048, **DPT_HEADS[kind])
        m.load_state_dict(synth_state_dict_like(m))
        preds, conf = m.to(DEV)(toks, images=images, patch_start_idx=5)
        assert rel_l2(preds.cpu().numpy(), g[f"{kind}_preds"]) < TOL, kind
        assert rel_l2(conf.cpu().numpy(), g[f"{kind}_conf"]) < TOL, kind


def test_unproject_matches_reference():
    from sailrecon_amd.utils.geometry import unproject_depth_map_to_point_map
    g = load_npz("g6_unproject.npz")
    pts = unproject_depth_map_to_point_map(torch.from_numpy(g["depth"]).to(DEV),
                                           torch.from_numpy(g["extrinsic"]).to(DEV),
                                           torch.from_numpy(g["intrinsic"]).to(DEV))
    assert isinstance(pts, np.ndarray) and pts.dtype == np.float64 and pts.shape == g["points"].shape
    assert rel_l2(pts, g["points"]) < 1e-5


def test_sailrecon_with_heads_end_to_end():
    """SailRecon with every head enabled (the reference's default constructor) at 224, N=2,
    fp32: result dicts carry the reference's keys and shapes, and the DPT outputs equal the
    oracle's DPT applied to this path's own aggregator features."""
    from oracle import sfm_oracle as O
    from sailrecon_amd.models.sail_recon import SailRecon
    from sailrecon_amd.utils.synth_weights import synth_state_dict_like
    torch.manual_seed(0)
    model = SailRecon(img_size=224)
    sd = synth_state_dict_like(model)
    model.load_state_dict(sd)
    model = model.to(DEV).eval()
    x = torch.rand(2, 3, 224, 224, generator=torch.Generator().manual_seed(1))
    images = torch.cat([x, x])[None].to(DEV)
    model.aggregator.generator.manual_seed(0)
    with torch.no_grad():
        res = model(images, no_reloc_list=[0, 1], reloc_list=[2, 3], fix_rank=300)
        model.aggregator.generator.manual_seed(0)  # same subsample draws as the forward above
        feats, psi, _ = model.aggregator(images, [0, 1], [2, 3], fix_rank=300)
    assert len(res) == 2
    keys = {"extrinsic", "intrinsic", "point_map_by_unprojection", "point_map", "rgbs", "xyz_cnf", "depth_map",
            "dpt_cnf", "cam_tokens", "images"}  # exactly the reference's (sail_recon.py:125-151)
    for r in res:
        assert set(r) == keys, sorted(r)
        assert r["extrinsic"].shape == (1, 3, 4) and r["intrinsic"].shape == (1, 3, 3)
        assert r["point_map"].shape == (1, 224, 224, 3) and r["xyz_cnf"].shape == (1, 224, 224)
        assert r["depth_map"].shape == (1, 224, 224, 1) and r["dpt_cnf"].shape == (1, 224, 224)
        assert isinstance(r["point_map_by_unprojection"], np.ndarray)
        assert r["point_map_by_unprojection"].shape == (1, 224, 224, 3)
        assert r["cam_tokens"].shape == (1, 2048) and r["images"].shape == (1, 3, 224, 224)
    toks = {l: feats[l].cpu() for l in (4, 11, 17, 23)}
    for kind, key, ckey in (("point", "point_map", "xyz_cnf"), ("depth", "depth_map", "dpt_cnf")):
        pre = f"{kind}_head."
        hsd = {k[len(pre):]: v for k, v in sd.items() if k.startswith(pre)}
        p_ref, c_ref = O.dpt_forward(hsd, "", toks, images[:, 2:].cpu(), psi,
                                     activation=DPT_HEADS[kind]["activation"],
                                     conf_activation=DPT_HEADS[kind]["conf_activation"])
        got = torch.stack([r[key][0] for r in res]).cpu()
        gotc = torch.stack([r[ckey][0] for r in res]).cpu()
        assert rel_l2(got.numpy(), p_ref[0].numpy()) < TOL, kind
        assert rel_l2(gotc.numpy(), c_ref[0].numpy()) < TOL, kind


@pytest.mark.parametrize("n,h,w,c,cout,stride,relu,resid", [
    (2, 19, 23, 64, 32, 1, False, False),
    (1, 37, 37, 128, 64, 2, False, False),     # resize_layers[3] shape class: 3x3 stride 2
    (2, 15, 11, 32, 36, 1, True, True),        # ResidualConvUnit conv2: ReLU on the input, += residual
    (1, 9, 130, 256, 4, 1, True, False),       # one image row spans several 128-pixel tiles
])
def test_conv3x3_implicit_gemm(n, h, w, c, cout, stride, relu, resid):
    """sr_conv3x3_f32 (implicit GEMM, the LDS-DMA gathers each tap's channel slice from the NHWC
    input, zero padding from a zero buffer) against fp64 F.conv2d; exact fp32 MFMA -> 1e-5."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import torch.nn.functional as F
    from sailrecon_amd import ops
    g = torch.Generator().manual_seed(n * 1000 + c)
    x = torch.randn(n, h, w, c, generator=g)
    wt = torch.randn(cout, c, 3, 3, generator=g) / (3 * c ** 0.5)
    b = torch.randn(cout, generator=g)
    xin = x.clamp_min(0) if relu else x
    ref = F.conv2d(xin.permute(0, 3, 1, 2).double(), wt.double(), b.double(), stride=stride, padding=1)
    ref = ref.permute(0, 2, 3, 1)
    ho, wo = ref.shape[1:3]
    base = torch.randn(n, ho, wo, cout, generator=g)
    if resid:
        ref = ref + base.double()
    out = base.clone().cuda() if resid else torch.empty(n, ho, wo, cout, device="cuda")
    wk = wt.permute(0, 2, 3, 1).reshape(cout, 9 * c).contiguous().cuda()
    ops.conv3x3(x.cuda(), wk, out, stride=stride, relu_in=relu, bias=b.cuda(),
                resid_gamma=torch.ones(cout, device="cuda") if resid else None)
    torch.cuda.synchronize()
    assert rel_l2(out.cpu().numpy(), ref.numpy()) < 1e-5
