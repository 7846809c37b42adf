"""Input formation on the HIP path: ImagePreprocessor (train/utils/io.py:10-195,
imc2021.py:260-301) and the load_fn loaders (sailrecon/utils/load_fn.py:13-240) against the
reference's own steps run with Pillow (goldens.pil_process_reference / pil_load_reference) and the
CPU oracle.  Integer resampling and exact divisions: the bar is bit-exact (torch.equal)."""

import numpy as np
import pytest
import torch

from goldens import pil_load_reference, pil_process_reference

pytestmark = pytest.mark.gpu
DEV = "cuda"
SIZES = [(300, 400), (640, 480), (518, 518), (97, 61), (1, 5), (1536, 2048), (700, 1000)]


def _rgb(hw, seed):
    return np.random.default_rng(seed).integers(0, 256, hw + (3,), dtype=np.uint8)


def _depth(hw, seed):
    # full uint16 range plus flat extremes: exercises Pillow's overshoot store (v % 256, v >> 8 clips)
    d = np.random.default_rng(seed).integers(0, 65536, hw, dtype=np.uint16)
    d[: hw[0] // 3] = 65535
    d[:, : hw[1] // 4] = 0
    return d


@pytest.mark.parametrize("hw", SIZES)
def test_preprocessor_bit_exact(hw):
    from PIL import Image
    from oracle import sfm_oracle as O
    from sailrecon_amd.utils.io import ImagePreprocessor
    pre = ImagePreprocessor(518, device=DEV)
    rgb, dep = _rgb(hw, 1), _depth(hw, 2)
    t, k2kp, kp2k = pre(Image.fromarray(rgb))
    ref = pil_process_reference(rgb, 518, False)
    assert t.is_cuda and t.shape == (1, 3, 518, 518) and t.dtype == torch.float32
    assert torch.equal(t.cpu(), ref)
    _, r1, r2 = O.preprocess_image(rgb, 518)
    assert torch.equal(k2kp, r1) and torch.equal(kp2k, r2)
    d, _, _ = pre.process_image_with_matrices(Image.fromarray(dep), is_depth=True)
    assert d.shape == (1, 1, 518, 518)
    assert torch.equal(d.cpu(), pil_process_reference(dep, 518, True))
    if hw[0] * hw[1] <= 400 * 400:
        assert torch.equal(d.cpu(), O.preprocess_image(dep, 518, is_depth=True)[0])


def test_to_tensor_bit_exact():
    from PIL import Image
    from sailrecon_amd.utils.io import ImagePreprocessor
    pre = ImagePreprocessor(518, device=DEV)
    rgb, dep = _rgb((123, 77), 3), _depth((123, 77), 4)
    t = pre.to_tensor(Image.fromarray(rgb))
    assert torch.equal(t.cpu(), torch.from_numpy(rgb).permute(2, 0, 1).float().div(255))
    d = pre.to_tensor(Image.fromarray(dep), is_depth=True)
    assert torch.equal(d.cpu(), torch.from_numpy(dep.astype(np.float32) / 1000)[None])


def test_process_views_scene_into_model_input():
    """A scene of mixed-size views formed straight into the anchor half of the 2N-frame input
    (imc2021.py:260-301 stacking, demo_imc_forward.py:76-82 duplication)."""
    from PIL import Image
    from sailrecon_amd.utils.io import ImagePreprocessor
    sizes = [(300, 400), (480, 640), (300, 400), (512, 512), (300, 400)]
    views = [_rgb(hw, 10 + i) for i, hw in enumerate(sizes)]
    pre = ImagePreprocessor(518, device=DEV)
    images = torch.empty(1, 2 * len(views), 3, 518, 518, device=DEV)
    out, k2kp, kp2k = pre.process_views([Image.fromarray(v) for v in views], out=images[0, :len(views)])
    images[0, len(views):] = images[0, :len(views)]
    assert k2kp.shape == (len(views), 3, 3) and kp2k.shape == (len(views), 3, 3)
    for i, v in enumerate(views):
        ref = pil_process_reference(v, 518, False)[0]
        assert torch.equal(images[0, i].cpu(), ref), i
        assert torch.equal(images[0, len(views) + i].cpu(), ref), i
    deps = [_depth(hw, 20 + i) for i, hw in enumerate(sizes)]
    d, _, _ = pre.process_views([Image.fromarray(x) for x in deps], is_depth=True)
    for i, x in enumerate(deps):
        assert torch.equal(d[i].cpu(), pil_process_reference(x, 518, True)[0]), i


def _pil_images():
    from PIL import Image
    rng = np.random.default_rng(7)
    ims = [Image.fromarray(_rgb((300, 400), 30)), Image.fromarray(_rgb((640, 480), 31)),
           Image.fromarray(_rgb((1000, 300), 32)), Image.fromarray(_rgb((200, 1000), 33)),
           Image.fromarray(rng.integers(0, 256, (250, 333), dtype=np.uint8)),  # 'L' -> RGB
           Image.fromarray(rng.integers(0, 256, (260, 270, 4), dtype=np.uint8), "RGBA")]  # blended onto white
    return ims


@pytest.mark.parametrize("mode", ["crop", "pad"])
def test_load_and_preprocess_images(mode):
    from sailrecon_amd.utils.load_fn import load_and_preprocess_images
    ims = _pil_images()
    got = load_and_preprocess_images(ims, mode=mode, device=DEV)
    ref = pil_load_reference(ims, mode=mode)
    assert got.shape == ref.shape
    assert torch.equal(got.cpu(), ref)
    one = load_and_preprocess_images(ims[:1], mode=mode, device=DEV)
    assert torch.equal(one.cpu(), pil_load_reference(ims[:1], mode=mode))


def test_load_and_preprocess_images_square():
    from sailrecon_amd.utils.load_fn import load_and_preprocess_images_square
    ims = _pil_images()
    got, coords = load_and_preprocess_images_square(ims, target_size=1024, device=DEV)
    ref, rcoords = pil_load_reference(ims, square_target=1024)
    assert torch.equal(got.cpu(), ref)
    assert torch.equal(coords, rcoords)


def test_wide_rows_and_steep_downscale_bit_exact():
    """Rows staged in LDS in bands of 1..8; a 7000-wide canvas (one row per band, 21 KB rows) and a
    tall one (7000 rows -> 518, 14:1 vertical)."""
    from PIL import Image
    from sailrecon_amd.utils.io import ImagePreprocessor
    pre = ImagePreprocessor(518, device=DEV)
    for hw in ((40, 7000), (7000, 33)):
        rgb = _rgb(hw, 41)
        t, _, _ = pre(Image.fromarray(rgb))
        assert torch.equal(t.cpu(), pil_process_reference(rgb, 518, False)), hw
        dep = _depth(hw, 42)
        d, _, _ = pre(Image.fromarray(dep), is_depth=True)
        assert torch.equal(d.cpu(), pil_process_reference(dep, 518, True)), hw


@pytest.mark.parametrize("hw", [(300, 400), (640, 480), (518, 518), (97, 61), (1536, 2048), (700, 1000)])
@pytest.mark.parametrize("is_depth", [False, True], ids=["rgb", "depth"])
def test_reverse_transform_tensor(hw, is_depth):
    """ImagePreprocessor.reverse_transform_tensor (io.py:197-259): the processed tensor back to the
    original size through the fused HIP resize + crop, against the oracle's restatement with the
    reference's own torch calls (F.interpolate bicubic / bilinear, align_corners=False, then the
    crop) on the host.  fp32 interpolation with a different summation order: 2e-6 rel-L2, 1e-4 max."""
    from oracle import sfm_oracle as O
    from sailrecon_amd.utils.io import ImagePreprocessor
    arr = _depth(hw, 11) if is_depth else _rgb(hw, 7)
    pre = ImagePreprocessor(518, device=DEV)
    t, _, kp2k = pre(arr, is_depth=is_depth)
    got = pre.reverse_transform_tensor(t[0], kp2k, 518, is_depth=is_depth)
    ref = O.reverse_transform_tensor(t[0].cpu(), kp2k, 518, is_depth=is_depth)
    torch.cuda.synchronize()
    assert tuple(got.shape) == tuple(ref.shape)
    rel = float((got.cpu().double() - ref.double()).norm() / ref.double().norm().clamp_min(1e-30))
    mx = float((got.cpu() - ref).abs().max())
    print(f"reverse_transform {hw} depth={is_depth}: out {tuple(got.shape)} rel {rel:.2e} max {mx:.2e}")
    assert rel < 2e-6 and mx < 1e-4 * max(1.0, float(ref.abs().max()))


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_reverse_transform_tensor_dtype(dtype):
    """reverse_transform_tensor keeps a reduced-precision input's dtype, as the reference's
    F.interpolate + slice do: the result equals the fp32 path rounded once, and matches
    the oracle's torch restatement on the same reduced-precision input within that rounding."""
    from oracle import sfm_oracle as O
    from sailrecon_amd.utils.io import ImagePreprocessor
    pre = ImagePreprocessor(518, device=DEV)
    t, _, kp2k = pre(_rgb((300, 400), 7))
    x = t[0].to(dtype)
    got = pre.reverse_transform_tensor(x, kp2k, 518)
    f32 = pre.reverse_transform_tensor(x.float(), kp2k, 518)
    torch.cuda.synchronize()
    assert got.dtype == dtype
    assert torch.equal(got, f32.to(dtype))
    ref = O.reverse_transform_tensor(x.float().cpu(), kp2k, 518)
    rel = float((got.cpu().double() - ref.double()).norm() / ref.double().norm())
    assert rel < (4e-3 if dtype == torch.bfloat16 else 6e-4), rel
