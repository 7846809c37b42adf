"""CPU checks of the framework's HOST orchestration (no GPU): the Aggregator /
CameraHead / pose-decode control flow — frame ordering, subsample row maps, token
positions, special tokens, output assembly — run with the C-ABI semantics implemented
in torch (tests/cpu_ops.py) and compared with the reference's golden vectors."""

import numpy as np
import pytest
import torch
import torch.nn as nn

import cpu_ops
from goldens import load_npz, rel_l2, rule_state_dict


class Hot(nn.Module):
    def __init__(self):
        super().__init__()
        from sailrecon_amd.heads.camera_head import CameraHead
        from sailrecon_amd.models.aggregator import Aggregator
        self.aggregator = Aggregator(img_size=56, patch_size=14, embed_dim=384, depth=2, num_heads=6,
                                     patch_embed="dinov2_vits14_reg", intermediate_layer_idx=[0, 1])
        self.camera_head = CameraHead(dim_in=768, trunk_depth=2, num_heads=6)


def small_model():
    torch.manual_seed(0)
    m = Hot().eval()
    m.load_state_dict(rule_state_dict("small_state_dict_keys.json"))
    return m


def test_state_dict_matches_reference_keys():
    import json
    from goldens import GOLDEN
    ref = json.load(open(f"{GOLDEN}/small_state_dict_keys.json"))
    mine = {k: list(v.shape) for k, v in Hot().state_dict().items()}
    assert mine == ref
    from sailrecon_amd.models.sail_recon import SailRecon
    ref = json.load(open(f"{GOLDEN}/state_dict_keys.json"))
    mine = {k: list(v.shape) for k, v in SailRecon(enable_point=False, enable_depth=False).state_dict().items()}
    assert mine == ref


@pytest.mark.parametrize("tag", ["56", "70"])
def test_host_logic_matches_reference(tag):
    from sailrecon_amd.utils.pose_enc import pose_encoding_to_extri_intri
    g = load_npz(f"g1_small_{tag}.npz")
    n = int(g["n_views"])
    images = torch.from_numpy(g["images"])
    m = small_model()
    m.aggregator.generator.manual_seed(0)
    with cpu_ops.installed(), torch.no_grad():
        feats, psi, cam_last = m.aggregator(images, list(range(n)), list(range(n, 2 * n)), fix_rank=int(g["fix_rank"]))
        poses = m.camera_head(feats, cam_last)
        ext, intr = pose_encoding_to_extri_intri(poses[-1], (images.shape[-2], images.shape[-1]))
    assert np.array_equal(m.aggregator.last_subsample_indices[:, 0].numpy(), g["sub_idx"])
    for layer in (0, 1):
        assert rel_l2(feats[layer].numpy(), g[f"feat_{layer}"]) < 1e-5
    assert rel_l2(cam_last.numpy(), g["cam_token_last_layer"]) < 1e-5
    assert rel_l2(np.stack([p.numpy() for p in poses]), g["pose_enc"]) < 1e-5
    assert rel_l2(ext.numpy(), g["extrinsic"]) < 1e-5


def test_non_canonical_lists_match_reference():
    """Anchors [3, 1, 4] / queries [0, 5, 2]: interleaved, permuted, frame 0 a query.  The host
    reordering path (internal order = no_reloc_list then reloc_list), the special-token types keyed
    on the ORIGINAL frame index (aggregator.py:287-299) and the output order are all compared
    value by value with the reference's own outputs (g11)."""
    g = load_npz("g11_small_interleaved.npz")
    images = torch.from_numpy(g["images"])
    no_reloc, reloc = g["no_reloc"].tolist(), g["reloc"].tolist()
    m = small_model()
    with cpu_ops.installed(), torch.no_grad():
        m.aggregator.generator.manual_seed(0)
        feats, _, cam = m.aggregator(images, no_reloc, reloc, fix_rank=int(g["fix_rank"]))
        poses = m.camera_head(feats, cam)
    assert np.array_equal(m.aggregator.last_subsample_indices[:, 0].numpy(), g["sub_idx"])
    for layer in (0, 1):
        assert rel_l2(feats[layer].numpy(), g[f"feat_{layer}"]) < 1e-5, layer
    assert rel_l2(cam.numpy(), g["cam_token_last_layer"]) < 1e-5
    assert rel_l2(np.stack([p.numpy() for p in poses]), g["pose_enc"]) < 1e-5


def test_bad_lists_raise():
    g = load_npz("g1_small_56.npz")
    images = torch.from_numpy(g["images"])
    m = small_model()
    with cpu_ops.installed(), pytest.raises(ValueError):
        m.aggregator(images, [0, 1, 2, 3], [0, 1, 2, 3], fix_rank=10)
    with cpu_ops.installed(), pytest.raises(ValueError):
        m.aggregator(images[:, :, :2], [0, 1], [2, 3], fix_rank=10)


def test_product_path_refuses_cpu_tensors():
    g = load_npz("g1_small_56.npz")
    m = small_model()
    with pytest.raises(RuntimeError, match="HIP path only"):
        m.aggregator(torch.from_numpy(g["images"]), [0, 1], [2, 3], fix_rank=10)


def test_deferred_residuals_equal_fused_epilogues(monkeypatch):
    """the proj residual folded into LN2 (SR_FUSED_RESID_LN) and the fc2
    residual deferred to the next LayerNorm over the same rows (SR_DEFER_RESID: DINO block i ->
    i + 1, the global / reloc blocks of layer l -> the frame block of layer l + 1 when no output
    map or camera-token copy reads x in between) give the same forward as the GEMMs' residual
    epilogues: the host bookkeeping of runtime.Pending (which rows, which gamma, applied once)."""
    from sailrecon_amd import ops, runtime
    from sailrecon_amd.heads.camera_head import CameraHead
    from sailrecon_amd.models.aggregator import Aggregator
    g = load_npz("g1_small_56_n5.npz")
    images = torch.from_numpy(g["images"])
    n = int(g["n_views"])
    torch.manual_seed(3)
    agg = Aggregator(img_size=56, patch_size=14, embed_dim=384, depth=4, num_heads=6,
                     patch_embed="dinov2_vits14_reg", intermediate_layer_idx=[1, 3]).eval()
    cam = CameraHead(dim_in=768, trunk_depth=2, num_heads=6).eval()
    for mod in (agg, cam):  # LayerScale gammas of 1e-2 would hide a mis-applied residual
        for name, prm in mod.named_parameters():
            if name.endswith(("gamma", "ls1.gamma", "ls2.gamma")):
                prm.data.uniform_(0.5, 1.5)
    outs = []
    orig = cpu_ops.residual_layernorm
    for on in (False, True):
        monkeypatch.setattr(runtime, "_DEFER_RESID", on)
        monkeypatch.setattr(runtime, "_FUSED_RESID_LN", on)
        monkeypatch.setattr(ops, "RESIDUAL_LN_COLS", ops.RESIDUAL_LN_COLS + ((384,) if on else ()))
        agg.generator.manual_seed(0)
        calls = []
        monkeypatch.setattr(cpu_ops, "residual_layernorm", lambda *a, **k: (calls.append(1), orig(*a, **k)))
        with cpu_ops.installed(), torch.no_grad():
            feats, _, cam_last = agg(images, list(range(n)), list(range(n, 2 * n)), fix_rank=int(g["fix_rank"]))
            poses = cam(feats, cam_last)
        # on: 11 DINO LN1s + 12 DINO LN2s + 3 x 4 aggregator LN2s + the frame LN1s of layers 1 and 3
        # (two row ranges each: anchors, queries) + the camera trunk's 2 blocks x 4 iterations of LN2
        assert len(calls) == (0 if not on else 11 + 12 + 3 * 4 + 2 * 2 + 8), len(calls)
        outs.append((feats[1].clone(), feats[3].clone(), cam_last.clone(), poses[-1].clone()))
    for a, b in zip(*outs):
        assert rel_l2(b.numpy(), a.numpy()) < 1e-6


def test_save_checkpoint_writes_flat_trained_weights(tmp_path):
    """train.step.save_checkpoint (train_imc.py:272-286): model_step_<k>.pt + model_latest.pt,
    weights only, holding the values in the trainer's flat fp32 buffer (parameters are views into
    it), loadable with torch.load(weights_only=True) and the reference's key names."""
    import torch
    from sailrecon_amd.train.params import FlatParams
    from sailrecon_amd.train.step import save_checkpoint
    from sailrecon_amd.layers.block import Block
    torch.manual_seed(0)
    m = Block(dim=128, num_heads=2, qk_norm=True, init_values=0.01)
    flat = FlatParams(m)
    flat.data.add_(0.5)  # an "optimizer step" on the flat buffer
    path = save_checkpoint(m, None, None, None, 7, 1.25, tmp_path / "ck")
    assert path.name == "model_step_7.pt" and (tmp_path / "ck" / "model_latest.pt").exists()
    sd = torch.load(path, weights_only=True)
    assert set(sd) == set(m.state_dict())
    for n, p in m.named_parameters():
        assert torch.equal(sd[n], flat.view(flat.data, n)), n

