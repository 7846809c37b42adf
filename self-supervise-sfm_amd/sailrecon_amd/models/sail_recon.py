"""SailRecon façade — drop-in for sailrecon/models/sail_recon.py:24-159.

``SailRecon(...).forward(views, no_reloc_list=None, reloc_list=None, fix_rank=300)``
returns one dict per query view, like the reference (sail_recon.py:153-159).  The
aggregator and camera head run on the HIP path; the DPT point/depth heads
 are separate modules that are only evaluated when enabled.
"""

from __future__ import annotations

import torch
import torch.nn as nn

from ..heads.camera_head import CameraHead
from ..utils.pose_enc import pose_encoding_to_extri_intri
from .aggregator import Aggregator, shard_range


class SailRecon(nn.Module):
    def __init__(self, img_size=518, patch_size=14, embed_dim=1024, enable_camera=True, enable_point=True,
                 enable_depth=True, enable_track=True, kv_cache=False):
        super().__init__()
        self.aggregator = Aggregator(img_size=img_size, patch_size=patch_size, embed_dim=embed_dim, kv_cache=kv_cache)
        self.camera_head = CameraHead(dim_in=2 * embed_dim) if enable_camera else None
        self.point_head = None
        self.depth_head = None
        if enable_point or enable_depth:
            from ..heads.dpt_head import DPTHead  # §8(f) rank 1
            if enable_point:
                self.point_head = DPTHead(dim_in=2 * embed_dim, output_dim=4, activation="inv_log",
                                          conf_activation="expp1")
            if enable_depth:
                self.depth_head = DPTHead(dim_in=2 * embed_dim, output_dim=2, activation="exp",
                                          conf_activation="expp1")
        self.cam_token_last_layer = None
        self.need_re_forward = False
        # opt-in extra result key: each view's 9-d pose encoding (the last camera-head iteration),
        # what train.loss.compute_loss differentiates; off by default so forward() returns exactly
        # the reference's keys (sail_recon.py:144-151)
        self.return_pose_enc = False

    def forward(self, views, no_reloc_list=None, reloc_list=None, fix_rank=300):
        rgbs = views if isinstance(views, torch.Tensor) else torch.cat([v["img"] for v in views], dim=0)
        if rgbs.dim() == 4:
            rgbs = rgbs.unsqueeze(0)
        if no_reloc_list is None:
            no_reloc_list = list(range(rgbs.shape[1]))
        if reloc_list is None:
            reloc_list = list(range(rgbs.shape[1]))
        rgb_feats, idx_patch, cam_token_last_layer = self.aggregator(rgbs, no_reloc_list, reloc_list,
                                                                     fix_rank=fix_rank)
        # frame-sharded aggregator (Aggregator.set_frame_sharding): this rank's query views only;
        # the camera head runs replicated on the gathered camera tokens of every view
        _, G, r = self.aggregator._world()
        q0, nq_l = shard_range(len(reloc_list), G, r)
        local_reloc = list(reloc_list)[q0:q0 + nq_l]
        if not local_reloc:  # more ranks than query views: this rank only served anchors
            return []
        # a list index is a blocking host->device copy of the index: it made the host wait for the
        # whole aggregator before enqueueing the heads.  Contiguous query frames (the demo's
        # reloc_list = range(N, 2N)) are a slice; others go through a pinned async index copy.
        if local_reloc and local_reloc == list(range(local_reloc[0], local_reloc[0] + len(local_reloc))):
            reloc_rgbs = rgbs[:, local_reloc[0]:local_reloc[0] + len(local_reloc)]
        else:
            idx = torch.tensor(local_reloc, dtype=torch.long).pin_memory().to(rgbs.device, non_blocking=True)
            reloc_rgbs = rgbs.index_select(1, idx)
        cam_tokens = rgb_feats[-1][:, :, 0]
        predictions = {}
        with torch.autocast("cuda", enabled=False):  # heads in fp32, sail_recon.py:118-119
            if self.camera_head is not None:
                cam_in = rgb_feats if G == 1 else [self.aggregator.last_query_cam_tokens[:, :, None]]
                cam_maps = self.camera_head(cam_in, cam_token_last_layer)
                pose = cam_maps[-1][:, q0:q0 + nq_l]
                extrinsic, intrinsic = pose_encoding_to_extri_intri(pose.contiguous(), (rgbs.shape[-2], rgbs.shape[-1]))
                predictions["extrinsic"] = extrinsic
                predictions["intrinsic"] = intrinsic
                if self.return_pose_enc:
                    predictions["pose_enc"] = pose
            if self.point_head is not None:
                xyz_map, xyz_cnf = self.point_head(rgb_feats, images=reloc_rgbs, patch_start_idx=idx_patch)
                predictions["point_map"] = xyz_map
                predictions["xyz_cnf"] = xyz_cnf
            if self.depth_head is not None:
                dpt_map, dpt_cnf = self.depth_head(rgb_feats, images=reloc_rgbs, patch_start_idx=idx_patch)
                predictions["depth_map"] = dpt_map
                predictions["dpt_cnf"] = dpt_cnf
                if self.camera_head is not None:
                    from ..utils.geometry import unproject_depth_map_to_point_map
                    pts = unproject_depth_map_to_point_map(dpt_map.squeeze(0), predictions["extrinsic"].squeeze(0),
                                                           predictions["intrinsic"].squeeze(0))
                    predictions["point_map_by_unprojection"] = pts[None]
        predictions["rgbs"] = reloc_rgbs
        predictions["cam_tokens"] = cam_tokens
        predictions["images"] = reloc_rgbs
        final_results = [{} for _ in range(len(local_reloc))]
        for key, value in predictions.items():
            for i in range(len(local_reloc)):
                final_results[i][key] = value[:, i]
        return final_results

    # ------------------------------------------------------------------ two-phase relocalisation
    def clear_cache(self):
        """sail_recon.py:161-174."""
        self.aggregator.clear_kv_cache()
        self.cam_token_last_layer = None
        self.need_re_forward = False

    @staticmethod
    def _views_to_rgbs(views):
        rgbs = views if isinstance(views, torch.Tensor) else torch.cat([v["img"] for v in views], dim=0)
        return rgbs.unsqueeze(0) if rgbs.dim() == 4 else rgbs

    def tmp_forward(self, views, no_reloc_list=None, reloc_list=[], fix_rank=300):  # noqa: B006 (reference)
        """Phase 1 (sail_recon.py:176-200): run the anchors once with kv_cache=True, keeping every
        layer's anchor-subsample K|V (in HBM) and the anchors' last-layer camera tokens."""
        if not self.aggregator.kv_cache:
            raise RuntimeError("tmp_forward needs SailRecon(kv_cache=True)")
        if reloc_list:
            raise NotImplementedError("tmp_forward with queries: the reference's cached attention returns zeros "
                                      "for them; relocalise queries with reloc()")
        if self.need_re_forward:
            self.aggregator.clear_kv_cache()
        else:
            self.need_re_forward = True
        rgbs = self._views_to_rgbs(views)
        if no_reloc_list is None:
            no_reloc_list = list(range(len(views)))
        _, _, cam_token_last_layer = self.aggregator(rgbs, no_reloc_list, [], fix_rank=fix_rank)
        if self.cam_token_last_layer is None:
            self.cam_token_last_layer = cam_token_last_layer.clone()

    def reloc(self, views, no_reloc_list=None, fix_rank=300, memory_save=True, save_depth=True, fast_reloc=False,
              ret_img=False):
        """Phase 2 (sail_recon.py:202-282): relocalise query views against the cached scene.
        Same flags and result keys as the reference; heads whose outputs the flags drop are not
        evaluated (the reference computes and discards them)."""
        rgbs = self._views_to_rgbs(views)
        rgb_feats, idx_patch = self.aggregator.forward_with_cache(rgbs, fix_rank=fix_rank)
        cam_tokens = rgb_feats[-1][:, :, 0]
        nviews = len(views)
        predictions = {}
        with torch.autocast("cuda", enabled=False):
            cam_maps = self.camera_head(rgb_feats, self.cam_token_last_layer)
            extrinsic, intrinsic = pose_encoding_to_extri_intri(cam_maps[-1].contiguous(),
                                                                (rgbs.shape[-2], rgbs.shape[-1]))
            predictions["extrinsic"] = extrinsic
            predictions["intrinsic"] = intrinsic
            if not fast_reloc:
                if not memory_save and self.point_head is not None:
                    xyz_map, xyz_cnf = self.point_head(rgb_feats, images=rgbs, patch_start_idx=idx_patch)
                if (save_depth or not memory_save) and self.depth_head is not None:
                    dpt_map, dpt_cnf = self.depth_head(rgb_feats, images=rgbs, patch_start_idx=idx_patch)
                if not memory_save:
                    from ..utils.geometry import unproject_depth_map_to_point_map
                    pts = unproject_depth_map_to_point_map(dpt_map.squeeze(0), extrinsic.squeeze(0),
                                                           intrinsic.squeeze(0))
                    predictions["point_map_by_unprojection"] = pts[None]
                    predictions["point_map"] = xyz_map
                    predictions["rgbs"] = rgbs
                    predictions["xyz_cnf"] = xyz_cnf
                if save_depth:
                    predictions["depth_map"] = dpt_map
                    predictions["dpt_cnf"] = dpt_cnf
                predictions["cam_tokens"] = cam_tokens
                if ret_img:
                    predictions["images"] = rgbs
        final_results = [{} for _ in range(nviews)]
        for key, value in predictions.items():
            for i in range(nviews):
                final_results[i][key] = value[:, i]
        return final_results
