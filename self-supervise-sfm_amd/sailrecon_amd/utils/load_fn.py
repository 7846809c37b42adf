"""Image loading for the model input — drop-in for sailrecon/utils/load_fn.py:13-240
(``load_and_preprocess_images_square``, ``load_and_preprocess_images``) with the resize, the
padding and ToTensor on the HIP path (Pillow-exact BICUBIC, utils/io.py).  Decoding, RGBA
compositing onto white and ``convert("RGB")`` stay on the host, as in the reference.  Returned
tensors are on ``device``; the warning for mixed shapes is printed like the reference's.
"""

from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np
import torch

from .io import MODE_8BIT, _pixels, _upload, resample_into


def _open_rgb(path):
    from PIL import Image
    img = Image.open(path) if not hasattr(path, "convert") else path
    if img.mode == "RGBA":
        background = Image.new("RGBA", img.size, (255, 255, 255, 255))
        img = Image.alpha_composite(background, img)
    return _pixels(img.convert("RGB"), False)


def load_and_preprocess_images_square(image_path_list: Sequence, target_size: int = 1024, device="cuda"
                                      ) -> Tuple[torch.Tensor, torch.Tensor]:
    """load_fn.py:13-96: centre-pad to a black square, BICUBIC to target_size, ToTensor; also the
    [x1, y1, x2, y2, width, height] of the original pixels in target space (host float32)."""
    if len(image_path_list) == 0:
        raise ValueError("At least 1 image is required")
    device = torch.device(device)
    out = torch.empty(len(image_path_list), 3, target_size, target_size, device=device)
    coords = []
    for i, p in enumerate(image_path_list):
        a = _open_rgb(p)
        h, w = a.shape[:2]
        m = max(w, h)
        left, top = (m - w) // 2, (m - h) // 2
        s = target_size / m
        coords.append(np.array([left * s, top * s, (left + w) * s, (top + h) * s, w, h]))
        resample_into(_upload([a], device), MODE_8BIT, (m, m), (left, top), (target_size, target_size),
                      out[i:i + 1])
    return out, torch.from_numpy(np.array(coords)).float()


def load_and_preprocess_images(image_path_list: Sequence, mode: str = "crop", device="cuda") -> torch.Tensor:
    """load_fn.py:99-240: "crop" = width 518, height rounded to a multiple of 14 and centre-cropped
    to 518; "pad" = longest side 518, other side a multiple of 14, padded to 518x518 with 1.0.
    Mixed shapes are padded (1.0, centred) to the largest height and width."""
    if len(image_path_list) == 0:
        raise ValueError("At least 1 image is required")
    if mode not in ["crop", "pad"]:
        raise ValueError("Mode must be either 'crop' or 'pad'")
    device = torch.device(device)
    T = 518
    plans: List[tuple] = []
    for p in image_path_list:
        a = _open_rgb(p)
        h, w = a.shape[:2]
        if mode == "pad" and w < h:
            nh, nw = T, round(w * (T / h) / 14) * 14
        else:
            nw, nh = T, round(h * (T / w) / 14) * 14
        row0, rows = 0, nh
        if mode == "crop" and nh > T:
            row0, rows = (nh - T) // 2, T
        fh, fw = (T, T) if mode == "pad" else (rows, nw)
        plans.append((a, nh, nw, row0, rows, fh, fw))
    shapes = {(pl[5], pl[6]) for pl in plans}
    if len(shapes) > 1:
        print(f"Warning: Found images with different shapes: {shapes}")
    H = max(s[0] for s in shapes)
    W = max(s[1] for s in shapes)
    out = torch.ones(len(plans), 3, H, W, device=device)
    for i, (a, nh, nw, row0, rows, fh, fw) in enumerate(plans):
        # offset of the resized pixels: pad-mode centring inside 518x518, then mixed-shape centring
        oy = (fh - rows) // 2 + (H - fh) // 2
        ox = (fw - nw) // 2 + (W - fw) // 2
        h, w = a.shape[:2]
        resample_into(_upload([a], device), MODE_8BIT, (h, w), (0, 0), (nh, nw),
                      out[i:i + 1, :, oy:oy + rows, ox:ox + nw], row0=row0)
    return out
