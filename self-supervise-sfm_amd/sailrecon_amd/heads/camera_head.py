"""CameraHead — MI355X-native re-design of sailrecon/heads/camera_head.py.

Same constructor, parameter names and ``forward(aggregated_tokens_list,
cam_token_last_layer, num_iterations=4)`` contract (camera_head.py:26-121).  Runs
in exact fp32 like the reference (autocast disabled, sail_recon.py:119):

  tokens = token_norm(cat(anchor cam tokens, query cam tokens))         :103-110
  per iteration                                                          :143-184
    embed_pose (9 -> C, small fp32 linear) -> SiLU -> poseLN_modulation GEMM
    adaLN (LayerNorm no-affine, eps 1e-6) * (1 + scale) + shift, * gate, + tokens
    trunk: 4 Blocks (fp32 GEMMs, fp32 attention with the camera mask: anchors see
           anchors, a query sees anchors + itself — build_lr_mask :197-228)
    pose_branch (fc1 GEMM + GELU, fc2 small linear) on trunk_norm
    pred += delta; activate_pose (T, quat linear; FoV ReLU)   head_act.py:12-60
"""

from __future__ import annotations

from typing import List

import torch
import torch.nn as nn

from .. import _lib, ops, runtime
from ..layers import Mlp
from ..layers.block import Block
from .head_act import activate_pose  # noqa: F401  (API mirror)


def build_lr_mask(S: int, no_reloc_list, device="cpu"):
    """camera_head.py:197-228 (True = masked), kept for API compatibility."""
    r_idx = torch.tensor([i for i in range(S) if i not in no_reloc_list], dtype=torch.long, device=device)
    l_idx = torch.as_tensor(no_reloc_list, dtype=torch.long, device=device).unique(sorted=True)
    mask = torch.zeros(S, S, dtype=torch.bool, device=device)
    if l_idx.numel() and r_idx.numel():
        mask[l_idx[:, None], r_idx[None, :]] = True
    if r_idx.numel() > 1:
        mask[r_idx[:, None], r_idx[None, :]] = True
        mask[r_idx, r_idx] = False
    return mask.unsqueeze(0).unsqueeze(0)


def modulate(x: torch.Tensor, shift: torch.Tensor, scale: torch.Tensor) -> torch.Tensor:
    return x * (1 + scale) + shift


class CameraHead(nn.Module):
    def __init__(self, dim_in: int = 2048, trunk_depth: int = 4, pose_encoding_type: str = "absT_quaR_FoV",
                 num_heads: int = 16, mlp_ratio: int = 4, init_values: float = 0.01, trans_act: str = "linear",
                 quat_act: str = "linear", fl_act: str = "relu"):
        super().__init__()
        if pose_encoding_type != "absT_quaR_FoV":
            raise ValueError(f"Unsupported camera encoding type: {pose_encoding_type}")
        if (trans_act, quat_act, fl_act) != ("linear", "linear", "relu"):
            raise NotImplementedError("only the reference defaults (linear, linear, relu) are on the hot path")
        self.target_dim = 9
        self.trans_act, self.quat_act, self.fl_act = trans_act, quat_act, fl_act
        self.trunk_depth = trunk_depth
        self.trunk = nn.Sequential(*[Block(dim=dim_in, num_heads=num_heads, mlp_ratio=mlp_ratio,
                                           init_values=init_values) for _ in range(trunk_depth)])
        self.token_norm = nn.LayerNorm(dim_in)
        self.trunk_norm = nn.LayerNorm(dim_in)
        self.empty_pose_tokens = nn.Parameter(torch.zeros(1, 1, self.target_dim))
        self.embed_pose = nn.Linear(self.target_dim, dim_in)
        self.poseLN_modulation = nn.Sequential(nn.SiLU(), nn.Linear(dim_in, 3 * dim_in, bias=True))
        self.adaln_norm = nn.LayerNorm(dim_in, elementwise_affine=False, eps=1e-6)
        self.pose_branch = Mlp(in_features=dim_in, hidden_features=dim_in // 2, out_features=self.target_dim, drop=0)
        self.dim_in = dim_in
        self.num_heads = num_heads
        self._ws = runtime.Workspace()

    def invalidate_packed(self):
        for blk in self.trunk:
            blk.invalidate_packed()

    def forward(self, aggregated_tokens_list, cam_token_last_layer: torch.Tensor, num_iterations: int = 4) -> List:
        tokens = aggregated_tokens_list[-1]
        dev = tokens.device
        runtime.require_device(tokens, "CameraHead")
        B, Nq = tokens.shape[0], tokens.shape[1]
        Na = cam_token_last_layer.shape[1]
        Sc = Na + Nq
        C = self.dim_in
        ws = self._ws
        f32 = torch.float32
        M = B * Sc
        # pose tokens = cat(anchor cam tokens, query cam tokens) -> token_norm   :103-110
        raw = ws.get("cam_raw", M, C, f32, dev)
        rv = raw.view(B, Sc, C)
        for b in range(B):  # the anchors' and the queries' camera tokens (row-strided) into one block
            ops.copy_rows(rv[b, :Na], cam_token_last_layer[b], Na)
            ops.copy_rows(rv[b, Na:], tokens[b, :, 0], Nq)
        tok = ws.get("cam_tok", M, C, f32, dev)
        ops.layernorm(raw, self.token_norm.weight, self.token_norm.bias, self.token_norm.eps, tok)

        pbs = [blk.packed(f32) for blk in self.trunk]
        hidden = pbs[0].w_fc1.shape[0]
        sc = runtime.scratch(ws, M, C, hidden, f32, dev, tag="_cam")
        emb = ws.get("cam_emb", M, C, f32, dev)
        act_emb = ws.get("cam_emb_silu", M, C, f32, dev)
        mod = ws.get("cam_mod", M, 3 * C, f32, dev)
        xn = ws.get("cam_xn", M, C, f32, dev)
        xm = ws.get("cam_x", M, C, f32, dev)
        hb = ws.get("cam_hb", M, C // 2, f32, dev)
        delta = ws.get("cam_delta", M, 9, f32, dev)
        pred = ws.get("cam_pred", M, 9, f32, dev)
        w_mod = self.poseLN_modulation[1].weight.detach().float().contiguous()
        b_mod = self.poseLN_modulation[1].bias.detach().float().contiguous()
        w_emb = self.embed_pose.weight.detach().float().contiguous()
        b_emb = self.embed_pose.bias.detach().float().contiguous()
        pbr = self.pose_branch
        outs = []
        for it in range(num_iterations):
            if it == 0:  # embed_pose(empty_pose_tokens) broadcast to every token, :145-146
                ops.linear_small(self.empty_pose_tokens.detach().float().reshape(1, 9).contiguous(), w_emb, b_emb,
                                 emb, rows=M, lda=0)
            else:  # embed_pose(pred.detach()), :148-150
                ops.linear_small(pred, w_emb, b_emb, emb, rows=M)
            ops.silu(emb, act_emb)
            ops.gemm(act_emb, w_mod, mod, _lib.SR_EPI_BIAS, bias=b_mod)
            ops.layernorm(tok, None, None, self.adaln_norm.eps, xn)
            ops.adaln_modulate(xn, tok, mod, xm)
            for pb in pbs:  # trunk with ~build_lr_mask, :163-166
                def attend(qkv, o, pb=pb):
                    for b in range(B):
                        r = slice(b * Sc, (b + 1) * Sc)
                        ops.attention(qkv[r, 0:C], qkv[r, C:2 * C], qkv[r, 2 * C:], o[r], heads=pb.heads,
                                      head_dim=pb.head_dim, batch=1, lq=Sc, q_bstride=0, l0=Sc, k0_bstride=0,
                                      mask_mode=_lib.SR_MASK_CAMERA, n_anchor=Na)
                runtime.run_block(pb, xm, 0, M, sc, attend, None)
            ops.layernorm(xm, self.trunk_norm.weight, self.trunk_norm.bias, self.trunk_norm.eps, xn)
            ops.gemm(xn, pbr.fc1.weight.detach().float().contiguous(), hb, _lib.SR_EPI_BIAS_GELU,
                     bias=pbr.fc1.bias.detach().float().contiguous())
            ops.linear_small(hb, pbr.fc2.weight.detach().float().contiguous(), pbr.fc2.bias.detach().float().contiguous(),
                             delta, rows=M)
            act = torch.empty(B, Sc, 9, device=dev, dtype=f32)
            ops.pose_update(pred, delta, act.view(M, 9), first=(it == 0))
            outs.append(act[:, Na:])
        return outs
