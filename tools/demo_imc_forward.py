#!/usr/bin/env python
"""The ``train/demo_imc_forward.py`` entry point (reference :25-143) on the MI355X-native path.

Flow, step for step with the reference:
  1. build ``SailRecon(kv_cache=False)`` (all heads, :29) and load a state_dict.  The reference
     fetches its checkpoint from a URL (:28-32); there is no network here, so ``--ckpt`` takes a
     local file, loaded with ``torch.load(..., weights_only=True)`` (nothing from the file is
     executed); without it the seeded synthetic weights of ``utils.synth_weights`` are used;
  2. per scene: N images -> [N, 3, 518, 518].  The reference reads IMC2021 HDF5 scenes (h5py and
     the data are absent); ``--images DIR`` forms a scene from image files with
     ``ImagePreprocessor.process_views`` (pad-to-square + Pillow-exact bicubic, io.py:75-153, the
     same transform IMC2021.__getitem__ applies), otherwise seeded U[0,1) images stand in;
  3. duplicate to 2N frames, anchors = first half, queries = second half (:74-82);
  4. ``model.forward(dup, no_reloc_list, reloc_list, fix_rank=300)`` under no_grad + bf16
     autocast (:92-101); the heads run in fp32 inside forward as in the reference;
  5. results to the host (eval.utils.device.to_cpu, :104) and the three outputs of :108-140:
     ``pred.ply`` (eval.utils.geometry.save_pointcloud_with_plyfile: the unprojected depth points
     coloured by the images), ``pred.txt`` (eval_utils.save_kitti_poses: camera-to-world = inverse of
     [extrinsic; 0 0 0 1], first three rows per line) and ``scene_info.txt``.  The ``eval`` package
     is absent from the reference, so the two writers are restated here from their call sites.

    python tools/demo_imc_forward.py [--ckpt sailrecon.pt] [--images DIR] [--num-images 5]
                                     [--scenes 1] [--out gpurun_out/demo_imc]
"""

from __future__ import annotations

import argparse
import os
import sys
from typing import Dict, List, Optional

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "self-supervise-sfm_amd"))

from sailrecon_amd.models.sail_recon import SailRecon  # noqa: E402


def to_cpu(x):
    """eval.utils.device.to_cpu (demo_imc_forward.py:11,104): nested dict/list of tensors -> host."""
    if isinstance(x, torch.Tensor):
        return x.detach().cpu()
    if isinstance(x, dict):
        return {k: to_cpu(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return type(x)(to_cpu(v) for v in x)
    return x


def save_pointcloud_ply(predictions: List[Dict], path: str) -> int:
    """Binary little-endian PLY of every view's ``point_map_by_unprojection`` (x, y, z float32)
    with the view's pixel colours (uchar r, g, b).  Returns the vertex count."""
    pts, cols = [], []
    for p in predictions:
        xyz = np.asarray(p["point_map_by_unprojection"]).reshape(-1, 3).astype(np.float32)
        rgb = p["images"]
        rgb = (rgb.float().numpy() if isinstance(rgb, torch.Tensor) else np.asarray(rgb)).reshape(3, -1).T
        ok = np.isfinite(xyz).all(1)
        pts.append(xyz[ok])
        cols.append(np.clip(rgb[ok] * 255.0 + 0.5, 0, 255).astype(np.uint8))
    xyz = np.concatenate(pts) if pts else np.zeros((0, 3), np.float32)
    rgb = np.concatenate(cols) if cols else np.zeros((0, 3), np.uint8)
    rec = np.empty(len(xyz), dtype=[("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("r", "u1"), ("g", "u1"), ("b", "u1")])
    rec["x"], rec["y"], rec["z"] = xyz[:, 0], xyz[:, 1], xyz[:, 2]
    rec["r"], rec["g"], rec["b"] = rgb[:, 0], rgb[:, 1], rgb[:, 2]
    with open(path, "wb") as f:
        f.write((f"ply\nformat binary_little_endian 1.0\nelement vertex {len(rec)}\n"
                 "property float x\nproperty float y\nproperty float z\n"
                 "property uchar red\nproperty uchar green\nproperty uchar blue\nend_header\n").encode())
        f.write(rec.tobytes())
    return len(rec)


def save_kitti_poses(poses_c2w: List[np.ndarray], path: str) -> None:
    """KITTI odometry format: one line per frame, the 3x4 top of the 4x4 pose, row-major."""
    with open(path, "w") as f:
        for T in poses_c2w:
            f.write(" ".join(f"{v:.9e}" for v in np.asarray(T)[:3, :4].reshape(-1)) + "\n")


def load_model(ckpt: Optional[str], device, img_size: int = 518, seed: int = 0) -> SailRecon:
    model = SailRecon(img_size=img_size, kv_cache=False)  # demo_imc_forward.py:29
    if ckpt:
        sd = torch.load(ckpt, map_location="cpu", weights_only=True)
        if isinstance(sd, dict) and "model" in sd and isinstance(sd["model"], dict):
            sd = sd["model"]  # train_imc.py:272-286 checkpoints wrap the state_dict
        model.load_state_dict(sd)
    else:
        from sailrecon_amd.utils.synth_weights import synth_state_dict_like
        torch.manual_seed(seed)
        model.load_state_dict(synth_state_dict_like(model))
    return model.to(device).eval()


def scene_images(images_dir: Optional[str], n: int, scene_idx: int, img_size: int, device) -> torch.Tensor:
    if images_dir:
        from PIL import Image
        from sailrecon_amd.utils.io import ImagePreprocessor
        names = sorted(f for f in os.listdir(images_dir)
                       if f.lower().endswith((".png", ".jpg", ".jpeg", ".bmp", ".tif", ".tiff")))
        names = names[scene_idx * n:(scene_idx + 1) * n]
        if not names:
            return torch.empty(0, 3, img_size, img_size, device=device)
        ims = [Image.open(os.path.join(images_dir, f)) for f in names]
        return ImagePreprocessor(target_size=img_size, device=device).process_views(ims)[0]
    g = torch.Generator().manual_seed(1000 + scene_idx)
    return torch.rand(n, 3, img_size, img_size, generator=g).to(device)


def demo(ckpt: Optional[str] = None, images_dir: Optional[str] = None, num_images: int = 5, max_scenes: int = 1,
         out_dir: str = "gpurun_out/demo_imc", img_size: int = 518, model: Optional[SailRecon] = None,
         verbose: bool = True) -> List[List[Dict]]:
    device = "cuda"
    if not torch.cuda.is_available():
        raise RuntimeError("demo_imc_forward runs on the HIP path (no ROCm device visible)")
    dtype = torch.bfloat16  # demo_imc_forward.py:22 (bf16 on every MI355X)
    log = print if verbose else (lambda *a, **k: None)
    if model is None:
        model = load_model(ckpt, device, img_size)
    results = []
    for scene_idx in range(max_scenes):
        images = scene_images(images_dir, num_images, scene_idx, img_size, device)
        if images.numel() == 0:
            log(f"no images for scene {scene_idx}, stopping")
            break
        n = images.shape[0]
        scene_name = f"scene{scene_idx:03d}"
        log(f"=== scene {scene_idx + 1}/{max_scenes}: {n} images {tuple(images.shape)}")
        duplicated = torch.cat([images, images], dim=0)  # :76
        no_reloc_list = list(range(n))                    # :81
        reloc_list = list(range(n, 2 * n))                # :82
        out = os.path.join(out_dir, f"scene_{scene_idx:03d}_{scene_name}_")
        os.makedirs(out, exist_ok=True)
        with torch.no_grad(), torch.autocast("cuda", dtype=dtype):  # :92-93
            predictions = model.forward(duplicated, no_reloc_list=no_reloc_list, reloc_list=reloc_list,
                                        fix_rank=300)  # :101
        predictions = [to_cpu(p) for p in predictions]  # :104
        nv = save_pointcloud_ply(predictions, os.path.join(out, "pred.ply"))  # :109-113
        w2c = [p["extrinsic"][0].float().numpy() for p in predictions]    # :118-120
        c2w = [np.linalg.inv(np.vstack([T, np.array([0, 0, 0, 1])])) for T in w2c]  # :121-124
        save_kitti_poses(c2w, os.path.join(out, "pred.txt"))              # :126-128
        with open(os.path.join(out, "scene_info.txt"), "w") as f:         # :131-138
            f.write(f"Scene Name: {scene_name}\n")
            f.write(f"Number of Images: {n}\n")
            f.write("Number of Correspondences: 0\n")
            f.write("Correspondence Pairs: []\n")
            f.write(f"Images Tensor Shape: {tuple(images.shape)}\n")
            f.write(f"Number of Predictions: {len(predictions)}\n")
        log(f"saved {nv} points, {len(c2w)} poses and the scene info under {out}")
        results.append(predictions)
    return results


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--ckpt", default=None, help="local SailRecon state_dict (.pt), loaded weights_only")
    ap.add_argument("--images", default=None, help="directory of scene images (N per scene, sorted)")
    ap.add_argument("--num-images", type=int, default=5)
    ap.add_argument("--scenes", type=int, default=1)
    ap.add_argument("--img-size", type=int, default=518)
    ap.add_argument("--out", default="gpurun_out/demo_imc")
    a = ap.parse_args(argv)
    demo(a.ckpt, a.images, a.num_images, a.scenes, a.out, a.img_size)


if __name__ == "__main__":
    main()
