"""Input formation on the HIP path — drop-in for train/utils/io.py:10-195 (ImagePreprocessor) as
used per view by train/datasets/imc2021.py:260-301.

Pad to a centred zero square, Pillow BICUBIC resize to ``target_size``, ToTensor (RGB / 255) or
uint16 depth / 1000, plus the K <-> K' matrices.  Decoding and mode conversion (``convert("RGB")``)
stay on the host like the reference; the pixels go to HBM as uint8 / uint16 and both resample
passes, the padding and the ToTensor scaling run in sr_pil_resample_h / sr_pil_resample_v_f32,
bit-exact with Pillow (tests/test_io_gpu.py).  Differences from the reference: tensors come back
on ``device`` (the K matrices stay on the host, float32, as in the reference), and
``process_views`` forms a whole scene at once (imc2021.py:260-301 stacking) with same-size views
in one launch pair.  ``reverse_transform_tensor`` (io.py:197-259, the evaluation helper that maps a
processed tensor back to the original image size) is one fused HIP launch (sr_resize_crop_chw_f32:
torch's align_corners=False bicubic / bilinear upsample with the padding crop folded in).
"""

from __future__ import annotations

from typing import Any, Dict, List, Sequence, Tuple, Union

import numpy as np
import torch

from .. import ops, runtime

Tensor = torch.Tensor
MODE_8BIT, MODE_I16 = 0, 1
_PREC = 22  # Pillow PRECISION_BITS
_TABLES: Dict[Tuple[int, int, int, str], Tuple[Tensor, Tensor]] = {}


def _bicubic(x: float) -> float:
    a = -0.5
    x = abs(x)
    if x < 1.0:
        return ((a + 2.0) * x - (a + 3.0)) * x * x + 1
    if x < 2.0:
        return (((x - 5) * x + 8) * x - 4) * a
    return 0.0


def pil_coeffs(in_size: int, out_size: int, mode: int) -> Tuple[np.ndarray, np.ndarray]:
    """Pillow's resample coefficients for one axis (Resample.c precompute_coeffs, bicubic,
    box = whole axis): bounds int32 [out, 2] = (first input index, taps) and weights [out, ksize]
    (int32 22-bit fixed point for 8-bit modes, float64 for 'I;16'; 0 past a column's taps)."""
    scale = in_size / out_size
    fs = max(scale, 1.0)
    support, ss = 2.0 * fs, 1.0 / fs
    ksize = int(np.ceil(support)) * 2 + 1
    bounds = np.zeros((out_size, 2), np.int32)
    kk = np.zeros((out_size, ksize), np.float64)
    for xx in range(out_size):
        center = (xx + 0.5) * scale
        xmin = max(int(center - support + 0.5), 0)
        xmax = min(int(center + support + 0.5), in_size) - xmin
        w = [_bicubic((x + xmin - center + 0.5) * ss) for x in range(xmax)]
        tot = sum(w)
        for x in range(xmax):
            kk[xx, x] = w[x] / tot if tot != 0.0 else w[x]
        bounds[xx] = (xmin, xmax)
    if mode == MODE_8BIT:
        kk = np.where(kk < 0, np.trunc(-0.5 + kk * (1 << _PREC)), np.trunc(0.5 + kk * (1 << _PREC))).astype(np.int32)
    return bounds, kk


def _fold_padding(bounds: np.ndarray, kk: np.ndarray, pad: int, extent: int) -> Tuple[np.ndarray, np.ndarray]:
    """Canvas table -> image table: the image occupies canvas [pad, pad + extent) and the rest of
    the canvas is 0, so taps outside it are dropped (Pillow adds 0 * weight for them: +-0, which
    leaves an integer or double sum unchanged) and the first index becomes image-relative."""
    b = np.zeros_like(bounds)
    k = np.zeros_like(kk)
    for o, (xmin, cnt) in enumerate(bounds):
        lo, hi = max(xmin, pad), min(xmin + cnt, pad + extent)
        if hi > lo:
            b[o] = (lo - pad, hi - lo)
            k[o, :hi - lo] = kk[o, lo - xmin:hi - xmin]
    return b, k


def _quad_major(bounds: np.ndarray, kk: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """[out, 2] / [out, ksize] -> [ceil(out/4), 2, 4] / [ceil(out/4), ksize, 4] (outputs past the
    end get no taps)."""
    out, ksize = kk.shape
    nq = (out + 3) // 4
    b = np.zeros((nq * 4, 2), np.int32)
    b[:out] = bounds
    c = np.zeros((nq * 4, ksize), kk.dtype)
    c[:out] = kk
    return (np.ascontiguousarray(b.reshape(nq, 4, 2).transpose(0, 2, 1)),
            np.ascontiguousarray(c.reshape(nq, 4, ksize).transpose(0, 2, 1)))


def pil_table(in_size: int, out_size: int, mode: int, device, quads: bool = False, pad: int = 0,
              extent: int = None) -> Tuple[Tensor, Tensor]:
    """Device tables for one axis of a canvas of ``in_size`` pixels holding the image at
    [pad, pad + extent) (zeros elsewhere), cached per shape.  ``quads``: the horizontal pass's
    quad-major layout.  Default pad/extent: the plain Pillow table of the whole axis."""
    extent = in_size if extent is None else extent
    key = (in_size, out_size, mode, str(device), quads, pad, extent)
    if key in _TABLES:
        return _TABLES[key]
    bounds, kk = pil_coeffs(in_size, out_size, mode)
    if pad != 0 or extent != in_size:
        bounds, kk = _fold_padding(bounds, kk, pad, extent)
    if quads:
        bounds, kk = _quad_major(bounds, kk)
    tab = (runtime.to_device(torch.from_numpy(bounds), device), runtime.to_device(torch.from_numpy(kk), device))
    _TABLES[key] = tab
    return tab


def _identity_table(n: int, mode: int, device, quads: bool = False) -> Tuple[Tensor, Tensor]:
    """One tap of weight 1 per output (ToTensor without resizing: both passes copy exactly)."""
    key = (-n, n, mode, str(device), quads)
    if key not in _TABLES:
        bounds = np.stack([np.arange(n, dtype=np.int32), np.ones(n, dtype=np.int32)], 1)
        coeffs = np.full((n, 1), 1 << _PREC, np.int32) if mode == MODE_8BIT else np.ones((n, 1), np.float64)
        if quads:
            bounds, coeffs = _quad_major(bounds, coeffs)
        _TABLES[key] = (runtime.to_device(torch.from_numpy(bounds), device),
                        runtime.to_device(torch.from_numpy(coeffs), device))
    return _TABLES[key]


def _pixels(image, is_depth: bool) -> np.ndarray:
    """Host decode step: PIL image (or array) -> uint8 [h, w, 3] RGB or uint16 [h, w] depth."""
    if is_depth:
        a = np.asarray(image)
        if a.dtype != np.uint16 or a.ndim != 2:
            raise ValueError(f"depth images must be uint16 'I;16' [h, w] (got {a.dtype} {a.shape})")
        return a
    if hasattr(image, "convert") and image.mode != "RGB":
        image = image.convert("RGB")
    a = np.asarray(image)
    if a.dtype != np.uint8 or a.ndim != 3 or a.shape[2] != 3:
        raise ValueError(f"RGB images must be uint8 [h, w, 3] (got {a.dtype} {a.shape})")
    return a


def _upload(arrays: Sequence[np.ndarray], device) -> Tensor:
    """Host pixels -> device [n, h, w, c] (uint8, or uint16 bits viewed as int16): one copy into a
    pinned staging buffer, then an async H2D on the current stream."""
    a0 = arrays[0]
    dt = torch.uint8 if a0.dtype == np.uint8 else torch.int16
    shape = (len(arrays),) + a0.shape + ((1,) if a0.ndim == 2 else ())
    if torch.device(device).type != "cuda":
        raise RuntimeError("sailrecon_amd input formation runs on the HIP path only (device must be a ROCm GPU)")
    buf = torch.empty(shape, dtype=dt, pin_memory=True)
    host = buf.numpy().view(a0.dtype).reshape((len(arrays),) + a0.shape)
    for i, a in enumerate(arrays):
        host[i] = a
    return buf.to(device, non_blocking=True)


def resample_into(pix: Tensor, mode: int, canvas: Tuple[int, int], pad: Tuple[int, int], size: Tuple[int, int],
                  out: Tensor, row0: int = 0) -> None:
    """pix [n, h, w, c] on device, pasted at pad=(left, top) into a zero canvas=(h, w), resized
    (Pillow BICUBIC) to size=(th_full, tw); output rows [row0, row0 + out.shape[2]) go to out
    [n, c, rows, tw] (fp32, strided) scaled by 1/255 (RGB) or 1/1000 (depth).  The canvas
    padding lives only in the tables (taps on it are dropped), so both passes touch image pixels only."""
    n, h, w, c = pix.shape
    ch_, cw_ = canvas
    th_full, tw = size
    bh, kh = pil_table(cw_, tw, mode, pix.device, quads=True, pad=pad[0], extent=w)
    bv, kv = pil_table(ch_, th_full, mode, pix.device, pad=pad[1], extent=h)
    div = 255.0 if mode == MODE_8BIT else 1000.0
    tmp = ops.pil_tmp(n, c, h, tw, pix.dtype, pix.device)
    ops.pil_resample_h(mode, pix, bh, kh, tw, tmp)
    ops.pil_resample_v(mode, tmp, bv[row0:], kv[row0:], div, out)


class ImagePreprocessor:
    """Mirror of train/utils/io.py:10-195 with the pixel work on the HIP path."""

    def __init__(self, target_size: int = 518, device: Union[str, torch.device] = "cuda"):
        self.target_size = target_size
        self.device = torch.device(device)

    def __call__(self, image, is_depth: bool = False) -> Tuple[Tensor, Tensor, Tensor]:
        return self.process_image_with_matrices(image, is_depth)

    def to_tensor(self, image, is_depth: bool = False) -> Tensor:
        """io.py:50-72: RGB -> [3, H, W] / 255, depth -> [1, H, W] / 1000 (fp32, on device)."""
        a = _pixels(image, is_depth)
        mode = MODE_I16 if is_depth else MODE_8BIT
        pix = _upload([a], self.device)
        _, h, w, c = pix.shape
        out = torch.empty(1, c, h, w, device=self.device)
        bh, kh = _identity_table(w, mode, self.device, quads=True)
        bv, kv = _identity_table(h, mode, self.device)
        tmp = ops.pil_tmp(1, c, h, w, pix.dtype, self.device)
        ops.pil_resample_h(mode, pix, bh, kh, w, tmp)
        ops.pil_resample_v(mode, tmp, bv, kv, 255.0 if mode == MODE_8BIT else 1000.0, out)
        return out[0]

    @staticmethod
    def _geometry(h: int, w: int) -> Tuple[int, int, int]:
        m = max(h, w)
        return m, (m - w) // 2, (m - h) // 2

    def process_image_with_matrices(self, image, is_depth: bool = False) -> Tuple[Tensor, Tensor, Tensor]:
        """io.py:75-153: ([1, C, T, T] fp32 on device, K_to_K_prime, K_prime_to_K)."""
        t, k2kp, kp2k = self.process_views([image], is_depth)
        return t, k2kp[0], kp2k[0]

    def process_views(self, images: Sequence, is_depth: bool = False, out: Tensor = None
                      ) -> Tuple[Tensor, Tensor, Tensor]:
        """A scene's views at once (imc2021.py:260-301): ([N, C, T, T], [N, 3, 3], [N, 3, 3]).
        ``out`` may be a caller-owned [N, C, T, T] fp32 slot (e.g. the first half of the
        aggregator's 2N-frame input)."""
        T = self.target_size
        mode = MODE_I16 if is_depth else MODE_8BIT
        arrays = [_pixels(im, is_depth) for im in images]
        c = 1 if is_depth else 3
        if out is None:
            out = torch.empty(len(arrays), c, T, T, device=self.device)
        if out.shape != (len(arrays), c, T, T):
            raise ValueError(f"process_views: out must be [{len(arrays)}, {c}, {T}, {T}]")
        runtime.require_device(out, "ImagePreprocessor")
        groups: Dict[Tuple[int, int], List[int]] = {}
        for i, a in enumerate(arrays):
            groups.setdefault(a.shape[:2], []).append(i)
        mats = [None] * len(arrays)
        for (h, w), idx in groups.items():
            m, pl, pt = self._geometry(h, w)
            pix = _upload([arrays[i] for i in idx], self.device)
            contiguous = idx == list(range(idx[0], idx[0] + len(idx)))
            dst = out[idx[0]:idx[0] + len(idx)] if contiguous else torch.empty(len(idx), c, T, T, device=self.device)
            resample_into(pix, mode, (m, m), (pl, pt), (T, T), dst)
            if not contiguous:
                out[idx] = dst
            s = T / m
            k = self._create_transformation_matrices({"scale_x": s, "scale_y": s, "offset_x": pl * s,
                                                      "offset_y": pt * s})
            for i in idx:
                mats[i] = k
        return out, torch.stack([k[0] for k in mats]), torch.stack([k[1] for k in mats])

    def reverse_transform_tensor(self, processed_tensor: Tensor, K_prime_to_K: Tensor, target_size: int,
                                 is_depth: bool = False) -> Tensor:
        """io.py:197-259: (C, target, target) back to the original (C, H, W).  The resize scale and
        padding come from K_prime_to_K exactly as the reference reads them (float32 .item() values,
        the same int() truncations); the bicubic (RGB) / bilinear (depth) upsample to max_side and the
        crop of the padding run as one launch on the tensor's device (no max_side^2 intermediate).
        The result has the input's dtype, as F.interpolate and the slice give it (a bf16 / fp16
        input is resampled in fp32 and rounded once at the end)."""
        runtime.require_device(processed_tensor, "ImagePreprocessor.reverse_transform_tensor")
        K = K_prime_to_K.detach().float().cpu()
        scale_x = 1.0 / K[0, 0].item()
        scale_y = 1.0 / K[1, 1].item()
        offset_x = -K[0, 2].item() * scale_x
        offset_y = -K[1, 2].item() * scale_y
        max_side = int(target_size / scale_x)
        pad_left = int(offset_x / scale_x)
        pad_top = int(offset_y / scale_y)
        width, height = max_side - 2 * pad_left, max_side - 2 * pad_top
        x = processed_tensor.float().contiguous()
        out = torch.empty(x.shape[0], height, width, device=x.device, dtype=torch.float32)
        ops.resize_crop_chw(x, max_side, pad_top, pad_left, out, bicubic=not is_depth)
        if processed_tensor.dtype != torch.float32:
            out = out.to(processed_tensor.dtype)
        return out

    def _create_transformation_matrices(self, transform_param: Dict[str, Any]) -> Tuple[Tensor, Tensor]:
        """io.py:155-195 (host, float32)."""
        sx, sy = transform_param["scale_x"], transform_param["scale_y"]
        ox, oy = transform_param["offset_x"], transform_param["offset_y"]
        k2kp = torch.tensor([[sx, 0.0, ox], [0.0, sy, oy], [0.0, 0.0, 1.0]], dtype=torch.float32)
        kp2k = torch.tensor([[1.0 / sx, 0.0, -ox / sx], [0.0, 1.0 / sy, -oy / sy], [0.0, 0.0, 1.0]],
                            dtype=torch.float32)
        return k2kp, kp2k
