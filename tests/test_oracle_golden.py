"""Pin the CPU oracle against golden vectors produced by the real reference.

These run on CPU only (no GPU, no HIP library) — they establish that
``oracle/sfm_oracle.py`` is a faithful restatement before it is trusted as the
checker for the HIP path.
"""

import numpy as np
import pytest
import torch

from goldens import SMALL_AGG, SMALL_CAM, load_npz, rel_l2, rule_state_dict
from oracle import sfm_oracle as O


def _run_small(tag):
    g = load_npz(f"g1_small_{tag}.npz")
    sd = rule_state_dict("small_state_dict_keys.json")
    n = int(g["n_views"])
    images = torch.from_numpy(g["images"])
    S = images.shape[1]
    n_patch = (images.shape[-1] // 14) ** 2
    rank = min(int(g["fix_rank"]), n_patch)
    gen = torch.Generator().manual_seed(0)
    sub = O.draw_subsample_indices(gen, 2, 1, n, n_patch, rank)
    assert np.array_equal(sub[:, 0].numpy(), g["sub_idx"]), "randperm replay order differs"
    out = O.hot_path_forward(sd, O.AggCfg(**SMALL_AGG), images, list(range(n)), list(range(n, S)),
                             int(g["fix_rank"]), sub, **SMALL_CAM)
    return g, out


@pytest.mark.parametrize("tag", ["56", "70"])
def test_small_end_to_end(tag):
    g, out = _run_small(tag)
    assert out["patch_start_idx"] == 5
    for layer in (0, 1):
        assert rel_l2(out["feats"][layer].numpy(), g[f"feat_{layer}"]) < 1e-5
    assert out["feats"][-1] is out["feats"][1]
    assert rel_l2(out["cam_token_last_layer"].numpy(), g["cam_token_last_layer"]) < 1e-5
    pe = np.stack([p.numpy() for p in out["pose_enc_list"]])
    assert rel_l2(pe, g["pose_enc"]) < 1e-5
    assert rel_l2(out["extrinsic"].numpy(), g["extrinsic"]) < 1e-5
    assert rel_l2(out["intrinsic"].numpy(), g["intrinsic"]) < 1e-5


def test_small_interleaved_lists():
    """Oracle on permuted + interleaved anchor/query lists (g11, reference-generated)."""
    g = load_npz("g11_small_interleaved.npz")
    sd = rule_state_dict("small_state_dict_keys.json")
    no_reloc, reloc = g["no_reloc"].tolist(), g["reloc"].tolist()
    images = torch.from_numpy(g["images"])
    gen = torch.Generator().manual_seed(0)
    sub = O.draw_subsample_indices(gen, 2, 1, len(no_reloc), 16, 10)
    assert np.array_equal(sub[:, 0].numpy(), g["sub_idx"])
    out = O.hot_path_forward(sd, O.AggCfg(**SMALL_AGG), images, no_reloc, reloc, 10, sub, **SMALL_CAM)
    for layer in (0, 1):
        assert rel_l2(out["feats"][layer].numpy(), g[f"feat_{layer}"]) < 1e-5
    assert rel_l2(out["cam_token_last_layer"].numpy(), g["cam_token_last_layer"]) < 1e-5
    pe = np.stack([p.numpy() for p in out["pose_enc_list"]])
    assert rel_l2(pe, g["pose_enc"]) < 1e-5


def test_block_kats():
    g = load_npz("g2_blocks.npz")
    sd = rule_state_dict("block_state_dict_keys.json", "agg")
    y = O.block(sd, "", torch.from_numpy(g["agg_x"]), 16, 1e-5, pos=torch.from_numpy(g["agg_pos"]),
                qk_norm=True, rope_base=100.0)
    assert rel_l2(y.numpy(), g["agg_y"]) < 1e-6
    sd = rule_state_dict("block_state_dict_keys.json", "dino")
    y = O.block(sd, "", torch.from_numpy(g["dino_x"]), 16, 1e-6)
    assert rel_l2(y.numpy(), g["dino_y"]) < 1e-6
    sd = rule_state_dict("block_state_dict_keys.json", "cam")
    y = O.block(sd, "", torch.from_numpy(g["cam_x"]), 16, 1e-5, mask=torch.from_numpy(g["cam_mask"]))
    assert rel_l2(y.numpy(), g["cam_y"]) < 1e-6


def test_op_kats():
    g = load_npz("g3_ops.npz")
    y = O.rope2d(torch.from_numpy(g["rope_in"]), torch.from_numpy(g["rope_pos"]), 100.0)
    assert rel_l2(y.numpy(), g["rope_out"]) < 1e-7
    allow = O.build_allow_block(4, [0, 1], [2, 3])
    assert np.array_equal(allow.numpy(), g["allow_4_2"])
    assert np.array_equal(allow.repeat_interleave(3, 0).repeat_interleave(3, 1).numpy(), g["allow_tok"])
    assert np.array_equal(O.build_lr_mask(6, [0, 1, 2]).numpy(), g["lr_mask_6_3"])


def _full(fname, tol):
    g = load_npz(fname)
    sd = rule_state_dict("state_dict_keys.json")
    n, img = int(g["n_views"]), int(g["img"])
    gen = torch.Generator().manual_seed(n)
    x = torch.rand(n, 3, img, img, generator=gen)
    images = torch.cat([x, x])[None]
    n_patch = (img // 14) ** 2
    sub = O.draw_subsample_indices(torch.Generator().manual_seed(0), 24, 1, n, n_patch, min(300, n_patch))
    assert np.array_equal(sub[:, 0].numpy(), g["sub_idx"])
    out = O.hot_path_forward(sd, O.AggCfg(), images, list(range(n)), list(range(n, 2 * n)), 300, sub)
    rows = torch.from_numpy(g["sample_rows"])
    for layer in (4, 11, 17, 23):
        v = out["feats"][layer][0]
        assert rel_l2(v.norm(dim=-1).numpy(), g[f"feat_{layer}_rownorm"]) < tol
        assert rel_l2(v[:, 0].numpy(), g[f"feat_{layer}_cam"]) < tol
        assert rel_l2(v.reshape(-1, v.shape[-1])[rows].numpy(), g[f"feat_{layer}_rows"]) < tol
    assert rel_l2(out["cam_token_last_layer"].numpy(), g["cam_token_last_layer"]) < tol
    pe = np.stack([p.numpy() for p in out["pose_enc_list"]])
    assert rel_l2(pe, g["pose_enc"]) < tol
    assert rel_l2(out["extrinsic"].numpy(), g["extrinsic"]) < tol
    assert np.isfinite(out["intrinsic"].numpy()).all()
    assert rel_l2(out["intrinsic"].numpy(), g["intrinsic"]) < tol


@pytest.mark.slow
def test_full_c1_224():
    _full("g4_c1_224.npz", 1e-5)


@pytest.mark.slow
def test_full_518_n1():
    _full("g5_518_n1.npz", 1e-5)


# ---------------------------------------------------------------- DPT heads (§8(f) rank 1)
@pytest.mark.parametrize("kind", ["point", "depth"])
def test_dpt_small_matches_reference(kind):
    from goldens import DPT_HEADS, DPT_SMALL, dpt_small_model_sd
    g = load_npz("g6_dpt_small.npz")
    _, sd = dpt_small_model_sd(kind)
    toks = {l: torch.from_numpy(g[f"tok_{l}"]) for l in DPT_SMALL["intermediate_layer_idx"]}
    preds, conf = O.dpt_forward(sd, "", toks, torch.from_numpy(g["images"]), 5,
                                layers=DPT_SMALL["intermediate_layer_idx"],
                                activation=DPT_HEADS[kind]["activation"],
                                conf_activation=DPT_HEADS[kind]["conf_activation"])
    assert rel_l2(preds.numpy(), g[f"{kind}_preds"]) < 1e-5
    assert rel_l2(conf.numpy(), g[f"{kind}_conf"]) < 1e-5


def test_dpt_feature_only_matches_reference():
    from goldens import DPT_SMALL, dpt_feat_model_sd
    g = load_npz("g6_dpt_feat_small.npz")
    _, sd = dpt_feat_model_sd()
    toks = {l: torch.from_numpy(g[f"tok_{l}"]) for l in DPT_SMALL["intermediate_layer_idx"]}
    feat = O.dpt_forward(sd, "", toks, torch.from_numpy(g["images"]), 5, layers=DPT_SMALL["intermediate_layer_idx"],
                         feature_only=True)
    assert feat.shape == g["feat"].shape
    assert rel_l2(feat.numpy(), g["feat"]) < 1e-5


def test_dpt_224_matches_reference():
    from goldens import DPT_HEADS, dpt_224_inputs, rule_state_dict
    g = load_npz("g6_dpt_224.npz")
    toks, images = dpt_224_inputs()
    for kind in ("point", "depth"):
        sd = rule_state_dict("dpt_state_dict_keys.json", kind)
        preds, conf = O.dpt_forward(sd, "", toks, images, 5, activation=DPT_HEADS[kind]["activation"],
                                    conf_activation=DPT_HEADS[kind]["conf_activation"])
        assert rel_l2(preds.numpy(), g[f"{kind}_preds"]) < 1e-5
        assert rel_l2(conf.numpy(), g[f"{kind}_conf"]) < 1e-5


def test_dpt_mirror_state_dict_keys_match_reference():
    """our DPTHead mirror has exactly the reference DPTHead's state_dict keys / shapes."""
    from goldens import DPT_HEADS, key_shapes
    from sailrecon_amd.heads.dpt_head import DPTHead
    for kind in ("point", "depth"):
        ours = sorted((k, tuple(v.shape)) for k, v in DPTHead(dim_in=2048, **DPT_HEADS[kind]).state_dict().items())
        assert ours == key_shapes("dpt_state_dict_keys.json", kind)


def test_unproject_matches_reference():
    g = load_npz("g6_unproject.npz")
    pts = O.unproject_depth(torch.from_numpy(g["depth"]), torch.from_numpy(g["extrinsic"]),
                            torch.from_numpy(g["intrinsic"]))
    assert rel_l2(pts.numpy(), g["points"]) < 1e-6


# ---------------------------------------------------------------- two-phase relocalisation (§8(f) rank 3)
@pytest.mark.slow
def test_kvcache_reloc_equals_one_pass_oracle():
    """The reference's tmp_forward + reloc(i) (g7, make_golden_kvcache.py) equals the one-pass
    forward with image i as the query frame (the generator also printed this); the oracle's
    one-pass hot path + DPT depth head reproduce it."""
    from goldens import DPT_HEADS
    g = load_npz("g7_kvcache.npz")
    sd = rule_state_dict("state_dict_keys.json")
    images = torch.from_numpy(g["images"])
    n = images.shape[0]
    n_patch = (images.shape[-1] // 14) ** 2
    i = 1
    sub = O.draw_subsample_indices(torch.Generator().manual_seed(0), 24, 1, n, n_patch, min(300, n_patch))
    frames = torch.cat([images, images[i:i + 1]])[None]
    out = O.hot_path_forward(sd, O.AggCfg(), frames, list(range(n)), [n], 300, sub)
    assert rel_l2(out["extrinsic"][0].numpy(), g[f"extrinsic_{i}"][0]) < 1e-5
    assert rel_l2(out["intrinsic"][0].numpy(), g[f"intrinsic_{i}"][0]) < 1e-5
    assert rel_l2(out["feats"][-1][0, :, 0].numpy(), g[f"cam_tokens_{i}"]) < 1e-5
    from goldens import key_shapes
    from sailrecon_amd.utils.synth_weights import synth_state_dict
    hsd = synth_state_dict(("depth_head." + k, s_) for k, s_ in key_shapes("dpt_state_dict_keys.json", "depth"))
    d, c = O.dpt_forward(hsd, "depth_head.", out["feats"], frames[:, n:], 5,
                         activation=DPT_HEADS["depth"]["activation"])
    assert rel_l2(d[0].numpy(), g[f"depth_map_{i}"]) < 1e-5
    assert rel_l2(c[0].numpy(), g[f"dpt_cnf_{i}"]) < 1e-5


# ---------------------------------------------------------------- input formation (§8(f) rank 2)
from goldens import pil_process_reference  # noqa: E402


@pytest.mark.parametrize("hw", [(300, 400), (97, 61), (518, 518), (640, 480), (1000, 777)])
def test_input_formation_oracle_bit_exact_vs_pil(hw):
    rng = np.random.default_rng(hw[0] * hw[1])
    rgb = rng.integers(0, 256, hw + (3,), dtype=np.uint8)
    dep = rng.integers(0, 65536, hw, dtype=np.uint16)
    t, k2kp, kp2k = O.preprocess_image(rgb, 518)
    assert torch.equal(t, pil_process_reference(rgb, 518, False))
    d, _, _ = O.preprocess_image(dep, 518, is_depth=True)
    assert torch.equal(d, pil_process_reference(dep, 518, True))
    K = torch.tensor([[500.0, 0, hw[1] / 2], [0, 510.0, hw[0] / 2], [0, 0, 1]])
    assert torch.allclose(kp2k @ (k2kp @ K), K, rtol=1e-6)


def test_input_formation_tables_match_oracle():
    """The host-built tables the HIP path uploads (utils/io.py pil_table) equal the oracle's
    restatement of Pillow's coefficients (8-bit fixed point and double)."""
    from sailrecon_amd.utils import io
    for i, o in ((1000, 518), (777, 518), (518, 518), (97, 518), (518, 1024), (1, 7)):
        b8, k8 = io.pil_table(i, o, io.MODE_8BIT, "cpu")
        b16, k16 = io.pil_table(i, o, io.MODE_I16, "cpu")
        assert torch.equal(b8, b16)
        for xx, (xmin, kk) in enumerate(O.pil_coeffs(i, o)):
            assert b8[xx].tolist() == [xmin, len(kk)]
            assert k8[xx, :len(kk)].tolist() == O.pil_fixed(kk)
            assert k16[xx, :len(kk)].tolist() == kk
            assert not k8[xx, len(kk):].any() and not k16[xx, len(kk):].any()
        for mode, k in ((io.MODE_8BIT, k8), (io.MODE_I16, k16)):  # quad-major layout of the h pass
            bq, kq = io.pil_table(i, o, mode, "cpu", quads=True)
            nq = (o + 3) // 4
            assert bq.shape == (nq, 2, 4) and kq.shape == (nq, k.shape[1], 4)
            assert torch.equal(bq.permute(0, 2, 1).reshape(-1, 2)[:o], b8)
            assert torch.equal(kq.permute(0, 2, 1).reshape(-1, k.shape[1])[:o], k)
            assert not bq.permute(0, 2, 1).reshape(-1, 2)[o:].any()


def test_transformation_matrices_match_reference_formula():
    from sailrecon_amd.utils.io import ImagePreprocessor
    pre = ImagePreprocessor(518, device="cpu")
    for h, w in ((300, 400), (640, 480), (518, 518)):
        m = max(h, w)
        pl, pt = (m - w) // 2, (m - h) // 2
        s = 518 / m
        k2kp, kp2k = pre._create_transformation_matrices({"scale_x": s, "scale_y": s, "offset_x": pl * s,
                                                         "offset_y": pt * s})
        _, r1, r2 = O.preprocess_image(np.zeros((h, w, 3), np.uint8), 518)
        assert torch.equal(k2kp, r1) and torch.equal(kp2k, r2)


def test_padding_folded_tables_equal_canvas_tables():
    """Dropping the taps that land on the zero padding (utils/io.py _fold_padding) gives the same
    integer and double sums as Pillow's pass over the padded canvas."""
    from sailrecon_amd.utils import io
    rng = np.random.default_rng(5)
    for canvas, extent, out in ((1024, 768, 518), (640, 480, 518), (97, 61, 518), (7000, 40, 518)):
        pad = (canvas - extent) // 2
        img = rng.integers(0, 65536, (3, extent)).astype(np.int64)
        full = np.zeros((3, canvas), np.int64)
        full[:, pad:pad + extent] = img
        for mode in (io.MODE_8BIT, io.MODE_I16):
            bc, kc = io.pil_coeffs(canvas, out, mode)
            bf, kf = io._fold_padding(bc, kc, pad, extent)
            for o in range(out):
                x0, n0 = bc[o]
                x1, n1 = bf[o]
                assert 0 <= x1 and x1 + n1 <= extent
                if mode == io.MODE_8BIT:
                    a = (full[:, x0:x0 + n0] * kc[o, :n0]).sum(1)
                    b = (img[:, x1:x1 + n1] * kf[o, :n1]).sum(1)
                    assert np.array_equal(a, b)
                else:
                    for r in range(3):
                        a = b = 0.0
                        for t in range(n0):
                            a += float(full[r, x0 + t]) * kc[o, t]
                        for t in range(kf.shape[1]):  # the kernel runs all taps (zeros past n1)
                            b += float(img[r, min(x1 + t, extent - 1)]) * kf[o, t]
                        assert a == b and np.signbit(a) == np.signbit(b)


@pytest.mark.parametrize("case", ["dummy", "shared", "multi"])
def test_oracle_imc_loss_matches_reference(golden_dir, case):
    """Oracle restatement of compute_loss + CDFLossIndexPytorch vs the reference modules
    (tests/golden/make_golden_loss.py): loss and d loss / d pose encoding."""
    import os

    import numpy as np
    from oracle import sfm_oracle as O
    z = np.load(os.path.join(golden_dir, "g8_loss.npz"))
    g = lambda k: torch.from_numpy(z[f"{case}/{k}"])  # noqa: E731
    enc = g("enc").clone().requires_grad_(True)
    n_nodes = int(max(g("nodes_src").max(), g("nodes_dst").max())) + 1
    loss = O.imc_loss(enc, (518, 518), g("kp2k"), bool(z[f"{case}/shared"]), g("src_idx"), g("dst_idx"),
                      g("src_coords"), g("dst_coords"), g("src_depth"), g("dst_depth"), g("nodes_src"),
                      g("nodes_dst"), n_nodes)
    loss.backward()
    assert abs(float(loss) - float(z[f"{case}/out_loss"])) <= 1e-6 * abs(float(z[f"{case}/out_loss"]))
    ref = g("out_grad")
    assert float((enc.grad - ref).norm() / ref.norm()) < 1e-5
