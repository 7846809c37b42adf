"""SailRecon training graph on the HIP path: aggregator + camera-head forward with saved
activations and the matching backward (the autograd graph that
``loss.backward()`` walks in train_imc.py:404 for predictions from sail_recon.py:70-159).

Scope: one scene per replica (B = 1, as train_imc.py's DataLoader batch_size=1 under DDP), the
aggregator in bf16 (autocast, train_imc.py:385) and the heads in fp32 (sail_recon.py:118-119).
The loss reaches the parameters only through the camera head's LAST iteration (the refinement
detaches the previous prediction, camera_head.py:148-150, and compute_loss reads
predictions[-1]), so the head keeps a tape for that iteration only; the DPT heads do not feed
the loss and get no gradient (DDP find_unused_parameters, train_imc.py:474).

Residual stream layout as in inference (models/aggregator.py): rows [0, Na*P) anchors,
[Na*P, S*P) queries, P = 5 + patches.  Backward walks the layers in reverse:

    layer l:  reloc block (query rows; its shared anchor-subsample segment's dK|dV -> the
              k-norm/RoPE backward -> K|V dgrad -> LayerNorm-through-row-map backward, added to
              the anchor rows) and global block (anchor rows) -> frame block (all rows)
    then the aggregator special tokens, DINO's final norm and blocks, the patch embedding.
"""

from __future__ import annotations

import os
from typing import Dict, List, Optional

import numpy as np
import torch

from .. import _lib, ops, runtime
from . import engine
from .params import FlatParams

Tensor = torch.Tensor
BF16 = torch.bfloat16
F32 = torch.float32
# SR_TRAIN_PAIR_DGRAD (default 1; 0 for the A/B): the layer's reloc and global blocks run their
# backward stage by stage with each stage's dgrad GEMMs grouped into one launch
_PAIR_DGRAD = os.environ.get("SR_TRAIN_PAIR_DGRAD", "1") != "0"
# SR_TRAIN_PAIR_FWD (default 1; 0 for the A/B): their forward likewise, each GEMM of the two
# blocks as one grouped launch (engine.run_block_train_multi)
_PAIR_FWD = os.environ.get("SR_TRAIN_PAIR_FWD", "1") != "0"


def _i32(rows, dev) -> Tensor:
    return runtime.to_device(torch.as_tensor(np.asarray(rows, dtype=np.int32)), dev)


class TrainGraph:
    """Training forward/backward for a SailRecon-style module with ``aggregator`` and
    ``camera_head`` (the DPT heads are not run: they do not feed the loss)."""

    def __init__(self, model, flat: Optional[FlatParams] = None, compute_dtype: torch.dtype = BF16):
        """``compute_dtype``: the aggregator's operand dtype.  bf16 (default) is train_imc.py's
        autocast; fp32 runs every aggregator GEMM and attention (forward and backward) in exact
        fp32, which pins the graph's wiring against fp32 autograd far below bf16 noise
        (tests/test_train_graph_gpu.py)."""
        if compute_dtype not in (BF16, F32):
            raise ValueError(f"TrainGraph: compute_dtype bf16 or fp32 (got {compute_dtype})")
        self.cdt = compute_dtype
        self.model = model
        self.agg = model.aggregator
        self.cam = model.camera_head
        self.flat = flat if flat is not None else FlatParams(model)
        self.dev = self.flat.data.device
        self.invalidate()
        self._tapes = {}
        self._sc = engine.BwdScratch()
        self._sc2 = engine.BwdScratch()  # the global block's scratch beside the reloc block's (block_bwd_multi)
        self.state: Optional[dict] = None
        # grad_ready_hook(module): called once a module's parameter grads are final within the
        # backward (data-parallel training starts that module's all-reduce right away)
        self.grad_ready_hook = None

    def _ready(self, module) -> None:
        if self.grad_ready_hook is not None:
            self.grad_ready_hook(module)

    # ------------------------------------------------------------------ parameter packs
    def invalidate(self) -> None:
        """Drop every derived weight pack (call after load_state_dict)."""
        self.agg.invalidate_packed()
        if self.cam is not None:
            self.cam.invalidate_packed()
        pe = self.agg.patch_embed
        if hasattr(pe, "_pos_cache"):
            pe._pos_cache = {}
        self._bwd: Dict[int, engine.BwdPack] = {}
        self._refresh_table = None  # (block keys, ops.weight_refresh_table) of refresh_packs
        self._packs_fresh = False

    def refresh_packs(self) -> None:
        """After an optimizer step: recast the bf16 forward weights in place (fp32 biases, gammas
        and norms alias the flat parameter buffer) and rebuild the transposed backward packs."""
        # bf16 blocks with a backward pack: every block's casts and transposed packs in ONE launch
        # (sr_weight_refresh_list_bf16 over a device table built once: the packs and the flat
        # parameter buffer do not move; one launch per block left the GPU waiting on the host)
        # (keyed on the pack objects, which the table's item list keeps alive: a re-created pack
        # rebuilds the table instead of refreshing a stale copy)
        blocks = [(self._bwd_src[k][0], self._bwd[k]) for k in self._bwd
                  if self._bwd_src[k][1] == BF16 and self._bwd_src[k][0]._packed.get(BF16) is not None]
        keys = tuple((id(blk), id(blk._packed[BF16]), id(into)) for blk, into in blocks)
        fused = {id(blk) for blk, _ in blocks}
        if keys:
            if self._refresh_table is None or self._refresh_table[0] != keys:
                items = []
                for blk, into in blocks:
                    items += engine.refresh_items_bf16(blk, blk._packed[BF16], into)
                self._refresh_table = (keys, ops.weight_refresh_table(items, self.dev), items)
            ops.weight_refresh_list(self._refresh_table[1])
        for blk in self._agg_blocks():
            pb = blk._packed.get(BF16)
            if pb is not None and id(blk) not in fused:
                a = blk.attn
                for src, dst in ((a.qkv.weight, pb.w_qkv), (a.proj.weight, pb.w_proj),
                                 (blk.mlp.fc1.weight, pb.w_fc1), (blk.mlp.fc2.weight, pb.w_fc2)):
                    ops.cast_bf16(src.detach(), dst)
        self.agg._packed.clear()  # patch weights / special-token table (small; rebuilt per step)
        pe = self.agg.patch_embed
        if hasattr(pe, "_pos_cache"):
            pe._pos_cache = {}
        for key in list(self._bwd):
            blk, dt = self._bwd_src[key]
            if id(blk) not in fused:
                engine.pack_bwd(blk, blk.packed(dt), dt, into=self._bwd[key])

    def _agg_blocks(self):
        a = self.agg
        out = list(a.frame_blocks) + list(a.global_blocks) + list(a.global_reloc_blocks)
        if hasattr(a.patch_embed, "blocks"):
            out += list(a.patch_embed.blocks)
        return out

    def _bwd_pack(self, blk, dt) -> engine.BwdPack:
        key = id(blk)
        if key not in self._bwd:
            if not hasattr(self, "_bwd_src"):
                self._bwd_src = {}
            self._bwd[key] = engine.pack_bwd(blk, blk.packed(dt), dt)
            self._bwd_src[key] = (blk, dt)
        return self._bwd[key]

    def _tape(self, key, rows, dim, hidden, dt, lse_numel, separate_raw) -> engine.BlockTape:
        t = self._tapes.get(key)
        if t is None or t.x0.shape[0] != rows or t.x0.shape[1] != dim or t.xn1.dtype != dt:
            t = engine.alloc_tape(rows, dim, hidden, dt, self.dev, lse_numel, separate_raw)
            self._tapes[key] = t
        return t

    def _buf(self, name, rows, cols, dt):
        return self._sc.get("g_" + name, rows, cols, dt, self.dev)

    # ------------------------------------------------------------------ forward
    def forward(self, images: Tensor, no_reloc_list: List[int], reloc_list: List[int], fix_rank=300) -> Tensor:
        """Training forward (aggregator bf16 + camera head fp32).  Returns the activated pose
        encoding of the query views of the last refinement iteration, [1, Nq, 9] (the
        ``pose_enc`` / extrinsic / intrinsic source of compute_loss), and keeps the tapes."""
        agg = self.agg
        B, S, C_in, H, W = images.shape
        if B != 1:
            raise NotImplementedError("training runs one scene per replica (B == 1, train_imc.py:503-510)")
        if C_in != 3:
            raise ValueError(f"Expected 3 input channels, got {C_in}")
        runtime.require_device(images, "TrainGraph")
        if sorted(list(no_reloc_list) + list(reloc_list)) != list(range(S)):
            raise ValueError("no_reloc_list and reloc_list must be disjoint and cover every frame")
        Na, Nq = len(no_reloc_list), len(reloc_list)
        if Na == 0 or Nq == 0:
            raise ValueError("training needs anchors and queries")
        ps = agg.patch_size
        assert H % ps == 0 and W % ps == 0
        dev = self.dev
        C, nh = agg.embed_dim, agg.num_heads
        gh, gw = H // ps, W // ps
        n_patch = gh * gw
        psi = agg.patch_start_idx
        P = n_patch + psi
        R = S * P
        q0 = Na * P
        hidden = agg.frame_blocks[0].mlp.fc1.out_features
        order = list(no_reloc_list) + list(reloc_list)
        imgs = images[:, order].reshape(S, 3, H, W).float().contiguous()
        st = dict(S=S, Na=Na, Nq=Nq, H=H, W=W, P=P, R=R, q0=q0, C=C, gh=gh, gw=gw, n_patch=n_patch)

        # ---- patch embed (+ DINO), vision_transformer.py:242-307 / aggregator.py:267-274
        x = self._buf("x", R, C, F32)
        kpad = -(-3 * ps * ps // 64) * 64
        cdt = self.cdt
        misc = agg._pack_misc(cdt, kpad)
        cols = self._buf("im2col", S * n_patch, kpad, cdt)
        ops.im2col_normalize(imgs, ps, cols, kpad)
        is_dino = hasattr(agg.patch_embed, "blocks")
        if is_dino:
            dino = agg.patch_embed
            st["pos_resampled"] = dino.pos_resampled(H, W)
            if st["pos_resampled"]:
                # interpolate_pos_encoding (vision_transformer.py:206-240) of the live parameter, every
                # step (the optimizer updates it in place): a 5 MB table transform on the device;
                # backward() applies its adjoint to the patch rows' colsum
                pe = dino.pos_embed.detach()[0]
                pos_tab = torch.cat([pe[:1], dino.resample_patch_pos(pe[1:], H, W)], 0).contiguous()
            else:
                pos_tab = dino.pos_embed_for(H, W)
            row_add = pos_tab[1:]
        else:
            row_add = self._buf("zeros_pos", n_patch, C, F32).zero_()
        ops.gemm(cols, misc["w_patch"], x, _lib.SR_EPI_PATCH, bias=misc["b_patch"], rows=S * n_patch,
                 patch=dict(seg_rows=n_patch, seg_stride=P, seg_offset=psi, row_add=row_add), tag="gemm")
        if is_dino:
            dtab = torch.cat([(dino.cls_token[0, 0] + pos_tab[0])[None], dino.register_tokens[0]], 0)
            ops.set_special_tokens(x, S, P, dtab.detach().float().contiguous()[None],
                                   torch.zeros(S, device=dev, dtype=torch.int32))
            for i, blk in enumerate(dino.blocks):
                pb = blk.packed(cdt)
                fwd, _ = engine.frame_attend_train(pb, S, P)
                engine.run_block_train(pb, x, 0, R, self._tape(("dino", i), R, C, hidden, cdt, S * pb.heads * P,
                                                                False), fwd, None)
            x_prenorm = self._buf("dino_prenorm", R, C, F32)
            ops.copy_rows(x_prenorm, x, R)
            ops.layernorm(x, dino.norm.weight, dino.norm.bias, dino.norm.eps, x)
        types = [0 if a == 0 else 1 for a in no_reloc_list] + [2] * Nq
        ops.set_special_tokens(x, S, P, misc["special"], _i32(types, dev))
        st["types"] = types

        # ---- subsample draws (aggregator.py:580-626), same generator order as inference
        agg.rank = min(fix_rank, n_patch) if fix_rank is not None else int(
            torch.randint(min(agg.min_rank, n_patch // 2), max(agg.min_rank, n_patch // 2), (1,),
                          generator=agg.generator).item())
        Pp = min(agg.rank + psi, P)
        idx = agg.draw_subsample(agg.depth, 1, Na, n_patch, agg.rank)
        agg.last_subsample_indices = torch.from_numpy(idx)
        base = (np.arange(Na) * P)[None, :, None]
        sel = base + psi + idx[:, 0]
        spec = np.broadcast_to(base + np.arange(psi)[None, None, :], (agg.depth, Na, psi))
        rowmap = np.concatenate([spec, sel], axis=-1).reshape(agg.depth, Na * Pp).astype(np.int32)
        rowmap_t = runtime.to_device(torch.from_numpy(rowmap), dev)
        n_sub = Na * Pp
        st.update(n_sub=n_sub, rowmap=rowmap_t)
        rope = agg.rope.tables(C // nh, max(gh, gw) + 1, dev) if agg.rope is not None else None
        posctx = dict(tokens_per_frame=P, patch_start=psi, grid_w=gw)
        st.update(rope=rope, posctx=posctx)

        # ---- alternating layers, aggregator.py:339-423
        Mc = S
        cam_in = self._buf("cam_in", Mc, 2 * C, F32)
        cam_rows = _i32([f * P for f in range(S)], dev)
        st["cam_rows"] = cam_rows
        for l in range(agg.depth):
            pf = agg.frame_blocks[l].packed(cdt)
            fwd, _ = engine.frame_attend_train(pf, S, P)
            engine.run_block_train(pf, x, 0, R, self._tape(("frame", l), R, C, hidden, cdt, S * pf.heads * P, True),
                                   fwd, runtime.qkv_params(pf, rope, pos_row_base=0, **posctx))
            if l == agg.depth - 1:
                ops.copy_rows(cam_in[:, :C], x, S, rowmap=cam_rows)
            pr = agg.global_reloc_blocks[l].packed(cdt)
            pg = agg.global_blocks[l].packed(cdt)
            # anchor-subsample K|V of the reloc block (reads the anchors before the global block)
            xn_sub = self._buf(f"xn_sub{l}", n_sub, C, cdt)
            kv_sub = self._buf(f"kv_sub{l}", n_sub, 2 * C, cdt)
            kv_raw = self._buf(f"kv_raw{l}", n_sub, 2 * C, cdt)
            ops.layernorm(x, pr.ln1_w, pr.ln1_b, pr.eps, xn_sub, rowmap=rowmap_t[l], rows=n_sub)
            epi = runtime.qkv_params(pr, rope, pos_rowmap=rowmap_t[l], **posctx)
            if epi is None:
                ops.gemm(xn_sub, pr.w_qkv[C:], kv_sub, _lib.SR_EPI_BIAS, bias=_sl(pr.b_qkv, C, 3 * C), tag="gemm")
            else:
                epi["col_offset"] = C
                ops.gemm(xn_sub, pr.w_qkv[C:], kv_sub, _lib.SR_EPI_QKV, bias=_sl(pr.b_qkv, C, 3 * C), qkv=epi,
                         aux=kv_raw, tag="gemm")
            rfwd, _ = self._reloc_attn(pr, kv_sub, None, Nq, P, n_sub)
            rel = dict(pb=pr, x=x, r0=q0, r1=R, tape=self._tape(("reloc", l), R - q0, C, hidden, cdt,
                                                                Nq * pr.heads * P, True),
                       attend=rfwd, qkv_epi=runtime.qkv_params(pr, rope, pos_row_base=q0, **posctx))
            gfwd, _ = self._global_attn(pg, q0)
            glo = dict(pb=pg, x=x, r0=0, r1=q0, tape=self._tape(("global", l), q0, C, hidden, cdt, pg.heads * q0, True),
                       attend=gfwd, qkv_epi=runtime.qkv_params(pg, rope, pos_row_base=0, **posctx))
            if _PAIR_FWD:  # disjoint rows; the reloc block's anchor K|V was projected above
                engine.run_block_train_multi([rel, glo])
            else:
                for it in (rel, glo):
                    engine.run_block_train(it["pb"], it["x"], it["r0"], it["r1"], it["tape"], it["attend"],
                                           it["qkv_epi"])
            if l == agg.depth - 1:
                ops.copy_rows(cam_in[:, C:], x, S, rowmap=cam_rows)
        self.state = st
        # ---- camera head, fp32 (camera_head.py:85-186)
        return self._camera_forward(cam_in, Na, Nq)

    def _global_attn(self, pg, La):
        C = pg.dim

        def fwd(qkv, o, lse):
            # the tape's q|k|v has readable tail rows (engine.alloc_tape): the hand-scheduled sweep's
            # ragged variant covers L = 21,984 (C4); the key bound comes from the per-launch key scan
            # (the weights move every step)
            ops.attention(qkv[:, 0:C], qkv[:, C:2 * C], qkv[:, 2 * C:], o, heads=pg.heads, head_dim=pg.head_dim,
                          batch=1, lq=La, q_bstride=0, l0=La, k0_bstride=0, lse=lse, tag="attn_global",
                          tail_readable=True)

        def bwd(tape, dO, dqkv):
            q = tape.qkv
            ops.attention_bwd(q[:, 0:C], q[:, C:2 * C], q[:, 2 * C:], tape.o, tape.lse, dO, dqkv[:, 0:C],
                              dqkv[:, C:2 * C], dqkv[:, 2 * C:], engine._delta(dqkv.device, pg.heads * La),
                              heads=pg.heads, batch=1, lq=La, q_bstride=0, l0=La, k0_bstride=0, tag="attn_bwd_global")
        return fwd, bwd

    def _reloc_attn(self, pr, kv_sub, dkv_sub, Nq, P, n_sub):
        C = pr.dim

        def fwd(qkv, o, lse):
            ops.attention(qkv[:, 0:C], kv_sub[:, 0:C], kv_sub[:, C:2 * C], o, heads=pr.heads, head_dim=pr.head_dim,
                          batch=Nq, lq=P, q_bstride=P, l0=n_sub, k0_bstride=0, k1=qkv[:, C:2 * C],
                          v1=qkv[:, 2 * C:3 * C], l1=P, k1_bstride=P, lse=lse, tag="attn_reloc")

        def bwd(tape, dO, dqkv):
            q = tape.qkv
            ops.attention_bwd(q[:, 0:C], kv_sub[:, 0:C], kv_sub[:, C:2 * C], tape.o, tape.lse, dO, dqkv[:, 0:C],
                              dkv_sub[:, 0:C], dkv_sub[:, C:2 * C], engine._delta(dqkv.device, Nq * pr.heads * P),
                              heads=pr.heads, batch=Nq, lq=P, q_bstride=P, l0=n_sub, k0_bstride=0,
                              k1=q[:, C:2 * C], v1=q[:, 2 * C:3 * C], dk1=dqkv[:, C:2 * C], dv1=dqkv[:, 2 * C:],
                              l1=P, k1_bstride=P, tag="attn_bwd_reloc")
        return fwd, bwd

    # ------------------------------------------------------------------ camera head
    def _camera_forward(self, cam_in: Tensor, Na: int, Nq: int) -> Tensor:
        cam = self.cam
        M, Cc = cam_in.shape
        f = lambda t: t.detach()  # noqa: E731 (fp32 contiguous params alias the flat buffer)
        tok = self._buf("cam_tok", M, Cc, F32)
        ops.layernorm(cam_in, cam.token_norm.weight, cam.token_norm.bias, cam.token_norm.eps, tok)
        pbs = [blk.packed(F32) for blk in cam.trunk]
        hid = pbs[0].w_fc1.shape[0]
        emb = self._buf("cam_emb", M, Cc, F32)
        act_emb = self._buf("cam_act_emb", M, Cc, F32)
        mod = self._buf("cam_mod", M, 3 * Cc, F32)
        xn_ada = self._buf("cam_xn_ada", M, Cc, F32)
        xm = self._buf("cam_xm", M, Cc, F32)
        xm_out = self._buf("cam_xm_out", M, Cc, F32)
        xn_t = self._buf("cam_xn_t", M, Cc, F32)
        pre = self._buf("cam_pre", M, Cc // 2, F32)
        hb = self._buf("cam_hb", M, Cc // 2, F32)
        delta = self._buf("cam_delta", M, 9, F32)
        pred = self._buf("cam_pred", M, 9, F32)
        pred_in = self._buf("cam_pred_in", M, 9, F32)
        act = torch.empty(M, 9, device=self.dev, dtype=F32)
        w_emb, b_emb = f(cam.embed_pose.weight), f(cam.embed_pose.bias)
        w_mod, b_mod = f(cam.poseLN_modulation[1].weight), f(cam.poseLN_modulation[1].bias)
        pbr = cam.pose_branch
        n_it = 4
        for it in range(n_it):
            last = it == n_it - 1
            if it == 0:
                ops.linear_small(f(cam.empty_pose_tokens).reshape(1, 9), w_emb, b_emb, emb, rows=M, lda=0)
            else:
                ops.linear_small(pred, w_emb, b_emb, emb, rows=M)
                if last:  # embed_pose's input (the detached previous prediction), for its weight grad
                    ops.copy2d(pred_in, pred)
            ops.silu(emb, act_emb)
            ops.gemm(act_emb, w_mod, mod, _lib.SR_EPI_BIAS, bias=b_mod)
            ops.layernorm(tok, None, None, cam.adaln_norm.eps, xn_ada)
            ops.adaln_modulate(xn_ada, tok, mod, xm)
            for bi, pb in enumerate(pbs):
                fwd = self._cam_attn(pb, M, Na)[0]
                if last:
                    engine.run_block_train(pb, xm, 0, M, self._tape(("cam", bi), M, Cc, hid, F32, 0, False), fwd, None)
                else:
                    sc = runtime.scratch(self._sc.ws, M, Cc, hid, F32, self.dev, tag="_camfwd")
                    runtime.run_block(pb, xm, 0, M, sc, lambda qkv, o, fwd=fwd: fwd(qkv, o, None), None)
            if last:
                ops.copy_rows(xm_out, xm, M)
            ops.layernorm(xm, cam.trunk_norm.weight, cam.trunk_norm.bias, cam.trunk_norm.eps, xn_t)
            ops.gemm(xn_t, f(pbr.fc1.weight), hb, _lib.SR_EPI_BIAS_GELU, bias=f(pbr.fc1.bias), aux=pre)
            ops.linear_small(hb, f(pbr.fc2.weight), f(pbr.fc2.bias), delta, rows=M)
            ops.pose_update(pred, delta, act, first=(it == 0))
        self.state.update(cam_M=M, cam_Na=Na, cam_act=act)
        return act[Na:].view(1, Nq, 9)

    def _cam_attn(self, pb, M, Na):
        C, H, D = pb.dim, pb.heads, pb.head_dim

        def fwd(qkv, o, lse):
            ops.attention(qkv[:, 0:C], qkv[:, C:2 * C], qkv[:, 2 * C:], o, heads=H, head_dim=D, batch=1, lq=M,
                          q_bstride=0, l0=M, k0_bstride=0, mask_mode=_lib.SR_MASK_CAMERA, n_anchor=Na)

        def bwd(tape, dO, dqkv):
            q = tape.qkv
            ops.attention_bwd_small(q[:, 0:C], q[:, C:2 * C], q[:, 2 * C:], dO, dqkv[:, 0:C], dqkv[:, C:2 * C],
                                    dqkv[:, 2 * C:], heads=H, head_dim=D, mask_mode=_lib.SR_MASK_CAMERA, n_anchor=Na)
        return fwd, bwd

    # ------------------------------------------------------------------ backward
    def backward(self, d_pose: Tensor) -> None:
        """Accumulate into every parameter's .grad the gradient of <d_pose, pose> where pose is
        forward()'s output ([1, Nq, 9] activated pose encoding of the last iteration)."""
        st = self.state
        if st is None:
            raise RuntimeError("backward() needs a training forward() first")
        d_raw = self._camera_backward(d_pose.reshape(-1, 9).float().contiguous())
        self._ready(self.cam)
        self._aggregator_backward(d_raw)
        self.state = None

    def _camera_backward(self, d_act_q: Tensor) -> Tensor:
        cam = self.cam
        st = self.state
        M, Na = st["cam_M"], st["cam_Na"]
        Cc = cam.dim_in
        g = lambda p: p.grad  # noqa: E731
        f = lambda t: t.detach()  # noqa: E731
        pbr = cam.pose_branch
        # activate_pose backward (FoV ReLU; translation / quaternion linear), head_act.py:12-60;
        # pred_4 = pred_3.detach() + delta_4 -> d delta_4 = d pred_4 (anchor rows: no loss)
        dd = self._buf("cd_delta", M, 9, F32)
        ops.pose_act_bwd(dd, d_act_q, st["cam_act"], Na)
        hb, pre, xn_t = self._buf("cam_hb", M, Cc // 2, F32), self._buf("cam_pre", M, Cc // 2, F32), \
            self._buf("cam_xn_t", M, Cc, F32)
        ops.wgrad_small(dd, hb, g(pbr.fc2.weight), db=g(pbr.fc2.bias), accumulate=True)
        w2t = self._buf("cw2t", Cc // 2, 9, F32)
        ops.transpose(f(pbr.fc2.weight), w2t)
        dhb = self._buf("cd_hb", M, Cc // 2, F32)
        ops.linear_small(dd, w2t, None, dhb, rows=M)
        dpre = self._buf("cd_pre", M, Cc // 2, F32)
        ops.act_bwd(ops.ACT_GELU, pre, dhb, dpre)
        ops.wgrad_small(dpre, xn_t, g(pbr.fc1.weight), db=g(pbr.fc1.bias), accumulate=True)
        w1t = self._buf("cw1t", Cc, Cc // 2, F32)
        ops.transpose(f(pbr.fc1.weight), w1t)
        dxn = self._buf("cd_xn", M, Cc, F32)
        ops.gemm(dpre, w1t, dxn, _lib.SR_EPI_F32)
        dxm = self._buf("cd_xm", M, Cc, F32).zero_()
        ops.layernorm_bwd(self._buf("cam_xm_out", M, Cc, F32), dxn, cam.trunk_norm.weight, cam.trunk_norm.eps, dxm,
                          dw=g(cam.trunk_norm.weight), db=g(cam.trunk_norm.bias))
        # trunk blocks (fp32, camera mask), reverse
        for bi in reversed(range(len(cam.trunk))):
            blk = cam.trunk[bi]
            pb = blk.packed(F32)
            _, bwd = self._cam_attn(pb, M, Na)
            engine.block_bwd(pb, self._bwd_pack(blk, F32), engine.block_grads(blk), self._tapes[("cam", bi)], dxm,
                             None, bwd, None, self._sc, tag="cam")
        # adaLN: xm = gate * (LN(tok) * (1 + scale) + shift) + tok
        tok = self._buf("cam_tok", M, Cc, F32)
        dtok = self._buf("cd_tok", M, Cc, F32)
        ops.copy_rows(dtok, dxm, M)
        dxa = self._buf("cd_xn_ada", M, Cc, F32)
        dmod = self._buf("cd_mod", M, 3 * Cc, F32)
        ops.adaln_bwd(self._buf("cam_xn_ada", M, Cc, F32), self._buf("cam_mod", M, 3 * Cc, F32), dxm, dxa, dmod)
        ops.layernorm_bwd(tok, dxa, None, cam.adaln_norm.eps, dtok)
        lin = cam.poseLN_modulation[1]
        act_emb = self._buf("cam_act_emb", M, Cc, F32)
        ops.wgrad_small(dmod, act_emb, g(lin.weight), db=g(lin.bias), accumulate=True)
        wmt = self._buf("cwmt", Cc, 3 * Cc, F32)
        ops.transpose(f(lin.weight), wmt)
        dact = self._buf("cd_act_emb", M, Cc, F32)
        ops.gemm(dmod, wmt, dact, _lib.SR_EPI_F32)
        demb = self._buf("cd_emb", M, Cc, F32)
        ops.act_bwd(ops.ACT_SILU, self._buf("cam_emb", M, Cc, F32), dact, demb)
        ops.wgrad_small(demb, self._buf("cam_pred_in", M, 9, F32), g(cam.embed_pose.weight),
                        db=g(cam.embed_pose.bias), accumulate=True)
        # token_norm
        d_raw = self._buf("cd_raw", M, Cc, F32).zero_()
        ops.layernorm_bwd(self._buf("cam_in", M, Cc, F32), dtok, cam.token_norm.weight, cam.token_norm.eps, d_raw,
                          dw=g(cam.token_norm.weight), db=g(cam.token_norm.bias))
        return d_raw

    def _aggregator_backward(self, d_raw: Tensor) -> None:
        agg = self.agg
        st = self.state
        S, Na, Nq, P, R, q0, C = st["S"], st["Na"], st["Nq"], st["P"], st["R"], st["q0"], st["C"]
        n_sub, rowmap, rope, posctx = st["n_sub"], st["rowmap"], st["rope"], st["posctx"]
        cam_rows = st["cam_rows"]
        g = lambda p: p.grad  # noqa: E731
        cdt = self.cdt
        bf = cdt == BF16
        dx = self._buf("dx", R, C, F32).zero_()
        dxb = self._buf("dxb", R, C, BF16) if bf else None  # fp32 mode: dx itself is the GEMM operand
        # camera tokens of the last layer: second half = after the global / reloc blocks
        ops.scatter_rows(dx, cam_rows, d_raw[:, C:], accumulate=True)
        dkv_sub = self._buf("dkv_sub", n_sub, 2 * C, F32)
        dkv_raw = self._buf("dkv_raw", n_sub, 2 * C, BF16) if bf else dkv_sub
        dxn_sub = self._buf("dxn_sub", n_sub, C, F32)
        for l in reversed(range(agg.depth)):
            if bf:
                ops.cast_bf16(dx, dxb)
            br, bg = agg.global_reloc_blocks[l], agg.global_blocks[l]
            pr, pg = br.packed(cdt), bg.packed(cdt)
            kv_sub = self._buf(f"kv_sub{l}", n_sub, 2 * C, cdt)
            # reloc block (query rows); its shared segment's dK|dV land in dkv_sub
            _, rbwd = self._reloc_attn(pr, kv_sub, dkv_sub, Nq, P, n_sub)
            gr = engine.block_grads(br)
            # global block (anchor rows)
            _, gbwd = self._global_attn(pg, q0)
            tg = self._tapes[("global", l)]
            rel = dict(pb=pr, bp=self._bwd_pack(br, cdt), g=gr, tape=self._tapes[("reloc", l)], dx=dx[q0:],
                       dxb=dxb[q0:] if bf else None, attend_bwd=rbwd, qkv_epi=runtime.qkv_params(pr, rope, pos_row_base=q0, **posctx),
                       sc=self._sc, tag="reloc")
            glo = dict(pb=pg, bp=self._bwd_pack(bg, cdt), g=engine.block_grads(bg), tape=tg, dx=dx[:q0],
                       dxb=dxb[:q0] if bf else None, attend_bwd=gbwd, qkv_epi=runtime.qkv_params(pg, rope, pos_row_base=0, **posctx),
                       sc=self._sc2, tag="global")
            if _PAIR_DGRAD and Nq > 0:
                # the two blocks' dgrad GEMMs stage by stage as grouped launches (engine.block_bwd_multi)
                engine.block_bwd_multi([rel, glo], tag="pair")
            else:
                for it in (rel, glo):
                    engine.block_bwd(it["pb"], it["bp"], it["g"], it["tape"], it["dx"], it["dxb"], it["attend_bwd"],
                                     it["qkv_epi"], self._sc, tag=it["tag"])
            # anchor subsample: k-norm + RoPE backward -> K|V dgrad / wgrad -> LN1 (row map) backward
            epi = runtime.qkv_params(pr, rope, pos_rowmap=rowmap[l], **posctx)
            if epi is not None:
                epi["col_offset"] = C
            kv_raw = self._buf(f"kv_raw{l}", n_sub, 2 * C, cdt) if epi is not None else None
            if bf or epi is not None:  # fp32 without qk-norm / RoPE: dkv_raw is dkv_sub
                ops.qk_bwd(kv_raw, dkv_sub, dkv_raw, epi or dict(embed_dim=C, head_dim=64, col_offset=C), grads=gr.qkn,
                           bias_grad=_sl(gr.b_qkv, C, 3 * C) if bf and engine.QK_COLSUM else None)
            bp = self._bwd_pack(br, cdt)
            ops.gemm(dkv_raw, bp.wt_qkv[:, C:], dxn_sub, _lib.SR_EPI_F32, tag="reloc.dgrad")
            xn_sub = self._buf(f"xn_sub{l}", n_sub, C, cdt)
            if bf:  # (the k|v bias grad came out of qk_bwd)
                ops.gemm_wgrad(dkv_raw, xn_sub, gr.w_qkv[C:], accumulate=True, tag="reloc.wgrad")
                if not engine.QK_COLSUM:
                    ops.colsum(dkv_raw, _sl(gr.b_qkv, C, 3 * C), accumulate=True)
            else:
                ops.wgrad_small(dkv_raw, xn_sub, gr.w_qkv[C:], db=_sl(gr.b_qkv, C, 3 * C), accumulate=True)
            ops.layernorm_bwd(tg.x0, dxn_sub, pr.ln1_w, pr.eps, dx, rowmap=rowmap[l], rows=n_sub,
                              dw=gr.ln1_w, db=gr.ln1_b)
            self._ready(br)
            self._ready(bg)
            if l == agg.depth - 1:  # first half of the camera tokens = the frame block's output
                ops.scatter_rows(dx, cam_rows, d_raw[:, :C], accumulate=True)
            if bf:
                ops.cast_bf16(dx, dxb)
            bf_ = agg.frame_blocks[l]
            pf = bf_.packed(cdt)
            _, fbwd = engine.frame_attend_train(pf, S, P)
            engine.block_bwd(pf, self._bwd_pack(bf_, cdt), engine.block_grads(bf_), self._tapes[("frame", l)], dx,
                             dxb, fbwd, runtime.qkv_params(pf, rope, pos_row_base=0, **posctx), self._sc, tag="frame")
            self._ready(bf_)
        self._embed_backward(dx, dxb)

    def _embed_backward(self, dx: Tensor, dxb: Tensor) -> None:
        agg = self.agg
        st = self.state
        S, Na, P, R, C, n_patch = st["S"], st["Na"], st["P"], st["R"], st["C"], st["n_patch"]
        psi = agg.patch_start_idx
        g = lambda p: p.grad  # noqa: E731
        # aggregator special tokens (aggregator.py:287-299): type 0 = ORIGINAL frame 0 as an
        # anchor, 1 = other anchors, 2 = queries (the forward's st["types"], per internal frame);
        # their rows were overwritten, so nothing flows below them.  Runs of equal type are
        # column-summed as strided frame views.
        dst = {0: (agg.camera_token.grad[0, 0, 0], agg.register_token.grad[0, 0]),
               1: (agg.camera_token.grad[0, 1, 0], agg.register_token.grad[0, 1]),
               2: (agg.camera_token_reloc.grad[0, 0, 0], agg.register_token_reloc.grad[0, 0])}
        types = st["types"]
        groups, f0 = [], 0
        for f in range(1, S + 1):
            if f == S or types[f] != types[f0]:
                groups.append((f0, f) + dst[types[f0]])
                f0 = f
        for f0, f1, gcam, greg in groups:
            view = dx[f0 * P:]
            ops.colsum(view.as_strided((f1 - f0, C), (P * C, 1)), gcam, accumulate=True)
            ops.colsum(view[1:].as_strided((f1 - f0, 4 * C), (P * C, 1)), greg.reshape(-1), accumulate=True)
        spec_rows = _i32([f * P + t for f in range(S) for t in range(psi)], self.dev)
        zero = self._buf("zero_row", 1, C, F32).zero_()[0]
        ops.scatter_rows(dx, spec_rows, zero, accumulate=False)
        if hasattr(agg.patch_embed, "blocks"):
            dino = agg.patch_embed
            dx2 = self._buf("dx2", R, C, F32).zero_()
            ops.layernorm_bwd(self._buf("dino_prenorm", R, C, F32), dx, dino.norm.weight, dino.norm.eps, dx2, dxb=dxb,
                              dw=g(dino.norm.weight), db=g(dino.norm.bias))
            dx = dx2
            for i in reversed(range(len(dino.blocks))):
                blk = dino.blocks[i]
                pb = blk.packed(self.cdt)
                _, bwd = engine.frame_attend_train(pb, S, P)
                engine.block_bwd(pb, self._bwd_pack(blk, self.cdt), engine.block_grads(blk), self._tapes[("dino", i)],
                                 dx, dxb, bwd, None, self._sc, tag="dino")
                self._ready(blk)
            # cls + pos[0] (row 0), registers (rows 1..4), patches + pos[1:] (vision_transformer.py:242-259)
            ops.colsum(dx.as_strided((S, C), (P * C, 1)), dino.cls_token.grad.reshape(-1), accumulate=True)
            ops.colsum(dx.as_strided((S, C), (P * C, 1)), dino.pos_embed.grad[0, 0], accumulate=True)
            ops.colsum(dx[1:].as_strided((S, 4 * C), (P * C, 1)), dino.register_tokens.grad.reshape(-1),
                       accumulate=True)
            if st.get("pos_resampled"):
                # adjoint of the bicubic resampling: d(pos_embed[1:]) += R^T d(table[1:])
                dtab = self._buf("dpos_tab", n_patch, C, F32)
                ops.colsum(dx[psi:].as_strided((S, n_patch * C), (P * C, 1)), dtab.reshape(-1))
                H, W = st["H"], st["W"]
                with torch.enable_grad():
                    src = dino.pos_embed.detach()[0, 1:].clone().requires_grad_(True)
                    dsrc, = torch.autograd.grad(dino.resample_patch_pos(src, H, W), src, dtab)
                ops.copy2d(dino.pos_embed.grad[0, 1:], dsrc.contiguous(), accumulate=True)
            else:
                ops.colsum(dx[psi:].as_strided((S, n_patch * C), (P * C, 1)),
                           dino.pos_embed.grad[0, 1:].reshape(-1), accumulate=True)
            conv = dino.patch_embed.proj
        else:
            conv = agg.patch_embed.proj
        # patch conv as im2col GEMM: dW = dpatch^T cols, db = colsum(dpatch)
        prow = _i32([f * P + psi + p for f in range(S) for p in range(n_patch)], self.dev)
        dpatch = self._buf("dpatch", S * n_patch, C, F32)
        ops.copy_rows(dpatch, dx, S * n_patch, rowmap=prow)
        kk = 3 * agg.patch_size ** 2
        kpad = -(-kk // 64) * 64
        cols = self._buf("im2col", S * n_patch, kpad, self.cdt)
        wtmp = self._buf("dw_patch", C, kpad, F32)
        if self.cdt == BF16:
            dpb = self._buf("dpatch_b", S * n_patch, C, BF16)
            ops.cast_bf16(dpatch, dpb)
            if kpad % 128:
                raise NotImplementedError("patch wgrad needs the im2col width to be a multiple of 128")
            ops.gemm_wgrad(dpb, cols, wtmp, tag="patch.wgrad")
        else:
            ops.wgrad_small(dpatch, cols, wtmp)
        ops.copy2d(conv.weight.grad.reshape(C, kk), wtmp[:, :kk], accumulate=True)
        if conv.bias is not None:
            ops.colsum(dpatch, conv.bias.grad, accumulate=True)
        self._ready(None)  # every remaining parameter


def _sl(t, a, b):
    return None if t is None else t[a:b]
