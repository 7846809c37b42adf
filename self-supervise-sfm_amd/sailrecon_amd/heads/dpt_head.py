"""DPT point / depth head on the HIP path — drop-in for sailrecon/heads/dpt_head.py:22-349.

Same constructor, submodule names and ``state_dict`` keys as the reference (the nn.Conv2d /
nn.ConvTranspose2d / nn.LayerNorm members only hold parameters; their forward is never used).
The forward runs on device in fp32 (the reference runs its heads with autocast disabled,
sail_recon.py:118), with feature maps in NHWC:

    tokens --LN (row map skips the 5 special tokens)--> 1x1 conv (GEMM) -> + uv pos-embed
      -> resize: ConvTranspose k4 / k2 (GEMM + scatter) | identity | 3x3 stride-2 conv
    layer*_rn 3x3 convs (im2col + GEMM) -> refinenet4..1 (ResidualConvUnits: ReLU fused into
      im2col, residual via the GEMM's gamma*(acc+bias) epilogue with gamma = 1; bilinear
      align_corners resize; 1x1 out_conv)
    output_conv1 (3x3) -> bilinear to the image size -> + pos-embed -> output_conv2[0] (3x3)
    -> ReLU + 1x1 + activate_head fused (sr_dpt_head_out_f32)

Frames are processed in chunks sized to bound the largest im2col buffer; results do not
depend on the chunking (every op is per frame), exactly as for the reference's
frames_chunk_size.
"""

from __future__ import annotations

from typing import Dict, List, Tuple, Union

import torch
import torch.nn as nn

from .. import _lib, ops, runtime

Tensor = torch.Tensor

IM2COL_BUDGET = 2 << 30  # bytes: largest im2col buffer per chunk (convs with C % 32 != 0 only)
ACT_BUDGET = 16 << 30    # bytes: activations of one chunk of frames (implicit-GEMM convs)


class ResidualConvUnit(nn.Module):
    """dpt_head.py:437-487 (bn=False, groups=1).  The reference's activation is an in-place
    nn.ReLU applied to the unit's own input, so the unit computes
    relu(x) + conv2(relu(conv1(relu(x)))) and leaves relu(x) in the caller's tensor."""

    def __init__(self, features: int):
        super().__init__()
        self.conv1 = nn.Conv2d(features, features, kernel_size=3, stride=1, padding=1, bias=True)
        self.conv2 = nn.Conv2d(features, features, kernel_size=3, stride=1, padding=1, bias=True)


class FeatureFusionBlock(nn.Module):
    """dpt_head.py:490-565 (deconv=False, bn=False, expand=False, align_corners=True)."""

    def __init__(self, features: int, has_residual: bool = True):
        super().__init__()
        self.out_conv = nn.Conv2d(features, features, kernel_size=1, stride=1, padding=0, bias=True)
        if has_residual:
            self.resConfUnit1 = ResidualConvUnit(features)
        self.has_residual = has_residual
        self.resConfUnit2 = ResidualConvUnit(features)


def _make_scratch(in_shape: List[int], out_shape: int) -> nn.Module:
    """dpt_head.py:383-434 (groups=1, expand=False)."""
    scratch = nn.Module()
    for i, c in enumerate(in_shape[:4]):
        setattr(scratch, f"layer{i + 1}_rn", nn.Conv2d(c, out_shape, kernel_size=3, stride=1, padding=1, bias=False))
    return scratch


class DPTHead(nn.Module):
    def __init__(self, dim_in: int, patch_size: int = 14, output_dim: int = 4, activation: str = "inv_log",
                 conf_activation: str = "expp1", features: int = 256,
                 out_channels: List[int] = [256, 512, 1024, 1024],  # noqa: B006 (reference signature)
                 intermediate_layer_idx: List[int] = [4, 11, 17, 23],  # noqa: B006
                 pos_embed: bool = True, feature_only: bool = False, down_ratio: int = 1) -> None:
        super().__init__()
        if activation not in ops.DPT_ACT or conf_activation not in ops.DPT_CONF_ACT:
            raise ValueError(f"unsupported activation {activation!r} / {conf_activation!r}")
        self.patch_size = patch_size
        self.activation = activation
        self.conf_activation = conf_activation
        self.pos_embed = pos_embed
        self.feature_only = feature_only
        self.down_ratio = down_ratio
        self.intermediate_layer_idx = intermediate_layer_idx
        self.output_dim = output_dim

        self.norm = nn.LayerNorm(dim_in)
        self.projects = nn.ModuleList([nn.Conv2d(dim_in, oc, kernel_size=1, stride=1, padding=0)
                                       for oc in out_channels])
        self.resize_layers = nn.ModuleList([
            nn.ConvTranspose2d(out_channels[0], out_channels[0], kernel_size=4, stride=4, padding=0),
            nn.ConvTranspose2d(out_channels[1], out_channels[1], kernel_size=2, stride=2, padding=0),
            nn.Identity(),
            nn.Conv2d(out_channels[3], out_channels[3], kernel_size=3, stride=2, padding=1),
        ])
        self.scratch = _make_scratch(out_channels, features)
        self.scratch.stem_transpose = None
        self.scratch.refinenet1 = FeatureFusionBlock(features)
        self.scratch.refinenet2 = FeatureFusionBlock(features)
        self.scratch.refinenet3 = FeatureFusionBlock(features)
        self.scratch.refinenet4 = FeatureFusionBlock(features, has_residual=False)
        head_features_1, head_features_2 = features, 32
        if feature_only:  # dpt_head.py:123-126: no output_conv2, features out
            self.scratch.output_conv1 = nn.Conv2d(head_features_1, head_features_1, kernel_size=3, stride=1,
                                                  padding=1)
        else:
            self.scratch.output_conv1 = nn.Conv2d(head_features_1, head_features_1 // 2, kernel_size=3, stride=1,
                                                  padding=1)
            self.scratch.output_conv2 = nn.Sequential(
                nn.Conv2d(head_features_1 // 2, head_features_2, kernel_size=3, stride=1, padding=1),
                nn.ReLU(inplace=True),
                nn.Conv2d(head_features_2, output_dim, kernel_size=1, stride=1, padding=0),
            )
        self._packed: Dict[str, Tensor] = {}
        self._ones: Dict[int, Tensor] = {}

    # ------------------------------------------------------------------ weight packing
    def invalidate_packed(self) -> None:
        self._packed.clear()

    def _load_from_state_dict(self, *args, **kwargs):  # noqa: D401 - keep packs in sync with loads
        self._packed.clear()
        return super()._load_from_state_dict(*args, **kwargs)

    def _pk(self, name: str, fn) -> Tensor:
        t = self._packed.get(name)
        if t is None:
            t = fn().detach().float().contiguous()
            self._packed[name] = t
        return t

    def _conv_w(self, name: str, conv: nn.Conv2d) -> Tensor:
        """[Cout, Cin, kh, kw] -> GEMM weight [Cout, kh*kw*Cin] (K order ky, kx, ci)."""
        return self._pk(name, lambda: conv.weight.permute(0, 2, 3, 1).reshape(conv.weight.shape[0], -1))

    def _convt_w(self, name: str, conv: nn.ConvTranspose2d) -> Tensor:
        """[Cin, Cout, k, k] -> GEMM weight [(ky, kx, co), Cin]."""
        return self._pk(name, lambda: conv.weight.permute(2, 3, 1, 0).reshape(-1, conv.weight.shape[0]))

    def _pos_table(self, h: int, w: int, c: int, aspect: float, device) -> Tensor:
        """The positional embedding ratio * sincos(uv grid) (dpt_head.py:300-315) of one [h, w, c]
        map: identical for every frame, so it is computed once per shape (the same kernel on a
        zero map) and added by the producing op's epilogue."""
        key = ("pos", h, w, c, float(aspect), str(device))
        t = self._packed.get(key)
        if t is None:
            t = torch.zeros(1, h, w, c, device=device, dtype=torch.float32)
            ops.dpt_pos_embed_(t, aspect, 0.1)
            self._packed[key] = t
        return t

    def _ones_for(self, c: int, device) -> Tensor:
        t = self._ones.get(c)
        if t is None or t.device != device:
            t = torch.ones(c, device=device, dtype=torch.float32)
            self._ones[c] = t
        return t

    # ------------------------------------------------------------------ building blocks
    @staticmethod
    def _gemm(a: Tensor, w: Tensor, bias, out: Tensor, epi=_lib.SR_EPI_BIAS, gamma=None) -> None:
        ops.gemm(a, w, out, epi, bias=None if bias is None else bias.detach().float().contiguous(), gamma=gamma,
                 splits=1)

    def _conv3x3(self, x: Tensor, name: str, conv: nn.Conv2d, stride: int = 1, relu_in: bool = False,
                 out: Tensor = None, resid: bool = False) -> Tensor:
        """3x3 / pad 1 conv of NHWC x; resid: out += conv(x) (+ bias) instead of out = ...
        C % 32 == 0 (every conv of the default heads): implicit GEMM (sr_conv3x3_f32, nothing
        materialised); otherwise im2col + GEMM."""
        n, h, w, c = x.shape
        ho, wo = (h - 1) // stride + 1, (w - 1) // stride + 1
        cout = conv.weight.shape[0]
        if c % 32 == 0 and cout % 4 == 0:
            if out is None:
                out = torch.empty(n, ho, wo, cout, device=x.device, dtype=torch.float32)
            bias = None if conv.bias is None else self._pk(name + ".bias", lambda: conv.bias)
            ops.conv3x3(x, self._conv_w(name, conv), out, stride=stride, relu_in=relu_in, bias=bias,
                        resid_gamma=self._ones_for(cout, x.device) if resid else None, tag="dpt_conv3x3")
            return out
        cols = torch.empty(n * ho * wo, 9 * c, device=x.device, dtype=torch.float32)
        ops.im2col3x3(x, stride, relu_in, cols)
        cout = conv.weight.shape[0]
        if out is None:
            out = torch.empty(n, ho, wo, cout, device=x.device, dtype=torch.float32)
        wt = self._conv_w(name, conv)
        if resid:
            self._gemm(cols, wt, conv.bias, out.view(-1, cout), _lib.SR_EPI_BIAS_RESID,
                       gamma=self._ones_for(cout, x.device))
        else:
            self._gemm(cols, wt, conv.bias, out.view(-1, cout))
        return out

    def _conv1x1(self, x: Tensor, name: str, conv: nn.Conv2d) -> Tensor:
        n, h, w, c = x.shape
        cout = conv.weight.shape[0]
        out = torch.empty(n, h, w, cout, device=x.device, dtype=torch.float32)
        self._gemm(x.view(-1, c), self._conv_w(name, conv), conv.bias, out.view(-1, cout))
        return out

    def _rcu_(self, x: Tensor, name: str, rcu: ResidualConvUnit) -> Tensor:
        """x <- relu(x) + conv2(relu(conv1(relu(x)))) in place (dpt_head.py:470-487, in-place ReLU)."""
        ops.relu_(x)
        t = self._conv3x3(x, name + ".conv1", rcu.conv1)
        self._conv3x3(t, name + ".conv2", rcu.conv2, relu_in=True, out=x, resid=True)
        return x

    def _fusion(self, name: str, blk: FeatureFusionBlock, x0: Tensor, x1: Tensor = None,
                size: Tuple[int, int] = None) -> Tensor:
        """FeatureFusionBlock.forward (dpt_head.py:540-565)."""
        out = x0
        if blk.has_residual and x1 is not None:
            res = self._rcu_(x1, name + ".resConfUnit1", blk.resConfUnit1)
            ops.add_(res, out)  # output = xs[0] + res  (res buffer is not reused)
            out = res
        out = self._rcu_(out, name + ".resConfUnit2", blk.resConfUnit2)
        n, h, w, c = out.shape
        ho, wo = size if size is not None else (int(h * 2), int(w * 2))
        up = torch.empty(n, ho, wo, c, device=out.device, dtype=torch.float32)
        ops.resize_bilinear(out, up)
        return self._conv1x1(up, name + ".out_conv", blk.out_conv)

    # ------------------------------------------------------------------ forward
    def forward(self, aggregated_tokens_list: Union[List[Tensor], Dict[int, Tensor]], images: Tensor,
                patch_start_idx: int, frames_chunk_size: int = 8) -> Union[Tensor, Tuple[Tensor, Tensor]]:
        """dpt_head.py:151-229: returns (preds [B,S,H,W,output_dim-1], conf [B,S,H,W]) fp32, or with
        feature_only the fused feature map [B, S, features, H', W'] (dpt_head.py:286-287; an NCHW
        view of the NHWC map the kernels write, no copy).  ``frames_chunk_size`` is accepted for
        signature parity; chunking here is sized by memory."""
        B, S, _, H, W = images.shape
        runtime.require_device(images, "DPTHead")
        dev = images.device
        ph, pw = H // self.patch_size, W // self.patch_size
        n_patch = ph * pw
        frames = B * S
        oh, ow = int(ph * self.patch_size / self.down_ratio), int(pw * self.patch_size / self.down_ratio)
        f = self.scratch.layer1_rn.weight.shape[0]  # features
        if self.feature_only:
            preds = torch.empty(frames, oh, ow, f, device=dev, dtype=torch.float32)
            conf = None
        else:
            preds = torch.empty(B, S, H, W, self.output_dim - 1, device=dev, dtype=torch.float32)
            conf = torch.empty(B, S, H, W, device=dev, dtype=torch.float32)
        convs3 = [m for m in self.modules() if isinstance(m, nn.Conv2d) and m.kernel_size == (3, 3)]
        if all(m.in_channels % 32 == 0 and m.out_channels % 4 == 0 for m in convs3):
            # implicit-GEMM convs: the chunk is bounded by its activations (largest: the upsampled
            # output_conv1 map + output_conv2's hidden map at oh x ow, the refinenet1 maps at 8x)
            per_frame = oh * ow * (f // 2 + 2 * (f // 8)) * 4 + (8 * ph) * (8 * pw) * f * 4 * 3
            chunk = max(1, min(frames, ACT_BUDGET // per_frame))
        else:
            per_frame = max(oh * ow * 9 * (self.scratch.output_conv1.weight.shape[0]) * 4,
                            (4 * ph) * (4 * pw) * 9 * self.scratch.layer1_rn.weight.shape[1] * 4)
            chunk = max(1, min(frames, IM2COL_BUDGET // per_frame))
        toks = []
        for layer_idx in self.intermediate_layer_idx:
            t = aggregated_tokens_list[layer_idx]
            runtime.require_device(t, "DPTHead tokens")
            if t.shape[:2] != (B, S):
                raise ValueError(f"token map {layer_idx} has shape {tuple(t.shape)}, images [{B}, {S}, ...]")
            toks.append(t.detach().float().contiguous().view(-1, t.shape[-1]))
        P = aggregated_tokens_list[self.intermediate_layer_idx[0]].shape[2]
        with torch.no_grad():
            for f0 in range(0, frames, chunk):
                f1 = min(frames, f0 + chunk)
                if self.feature_only:
                    self._forward_chunk(toks, P, patch_start_idx, f0, f1, ph, pw, H, W, oh, ow, preds[f0:f1], None)
                else:
                    self._forward_chunk(toks, P, patch_start_idx, f0, f1, ph, pw, H, W, oh, ow,
                                        preds.view(frames, H, W, -1)[f0:f1], conf.view(frames, H, W)[f0:f1])
        if self.feature_only:
            return preds.view(B, S, oh, ow, f).permute(0, 1, 4, 2, 3)
        return preds, conf

    def _forward_chunk(self, toks, P, psi, f0, f1, ph, pw, H, W, oh, ow, preds, conf):
        dev = toks[0].device
        F_ = f1 - f0
        n_patch = ph * pw
        aspect = W / H
        rows = (torch.arange(f0, f1, device=dev, dtype=torch.int32)[:, None] * P + psi
                + torch.arange(n_patch, device=dev, dtype=torch.int32)[None, :]).reshape(-1).contiguous()
        feats = []
        for i, tok in enumerate(toks):
            C = tok.shape[1]
            xn = torch.empty(F_ * n_patch, C, device=dev, dtype=torch.float32)
            ops.layernorm(tok, self.norm.weight.detach().float(), self.norm.bias.detach().float(), self.norm.eps, xn,
                          rowmap=rows, rows=F_ * n_patch)
            proj = self.projects[i]
            oc = proj.weight.shape[0]
            y = torch.empty(F_, ph, pw, oc, device=dev, dtype=torch.float32)
            if self.pos_embed:  # projection + bias + the per-frame positional table in one epilogue
                ops.gemm(xn, self._conv_w(f"projects.{i}", proj), y.view(-1, oc), _lib.SR_EPI_PATCH,
                         bias=self._pk(f"projects.{i}.bias", lambda: proj.bias),
                         patch=dict(seg_rows=n_patch, seg_stride=n_patch, seg_offset=0,
                                    row_add=self._pos_table(ph, pw, oc, aspect, dev).view(n_patch, oc)),
                         splits=1)
            else:
                self._gemm(xn, self._conv_w(f"projects.{i}", proj), proj.bias, y.view(-1, oc))
            layer = self.resize_layers[i]
            if isinstance(layer, nn.ConvTranspose2d):
                k = layer.kernel_size[0]
                g = torch.empty(F_ * n_patch, k * k * oc, device=dev, dtype=torch.float32)
                self._gemm(y.view(-1, oc), self._convt_w(f"resize_layers.{i}", layer), None, g)
                out = torch.empty(F_, ph * k, pw * k, oc, device=dev, dtype=torch.float32)
                ops.convt_scatter(g, F_, ph, pw, k, oc, layer.bias.detach().float().contiguous(), out)
                y = out
            elif isinstance(layer, nn.Conv2d):
                y = self._conv3x3(y, f"resize_layers.{i}", layer, stride=2)
            feats.append(y)
        sc = self.scratch
        l1, l2, l3, l4 = (self._conv3x3(f, f"scratch.layer{i + 1}_rn", getattr(sc, f"layer{i + 1}_rn"))
                          for i, f in enumerate(feats))
        out = self._fusion("scratch.refinenet4", sc.refinenet4, l4, size=tuple(l3.shape[1:3]))
        out = self._fusion("scratch.refinenet3", sc.refinenet3, out, l3, size=tuple(l2.shape[1:3]))
        out = self._fusion("scratch.refinenet2", sc.refinenet2, out, l2, size=tuple(l1.shape[1:3]))
        out = self._fusion("scratch.refinenet1", sc.refinenet1, out, l1)
        out = self._conv3x3(out, "scratch.output_conv1", sc.output_conv1)
        up = preds if self.feature_only else torch.empty(F_, oh, ow, out.shape[3], device=dev, dtype=torch.float32)
        ops.resize_bilinear(out, up, add=self._pos_table(oh, ow, out.shape[3], aspect, dev) if self.pos_embed else None)
        if self.feature_only:  # dpt_head.py:286-287: the fused, upsampled, position-embedded map
            return
        c0, c2 = sc.output_conv2[0], sc.output_conv2[2]
        hidden = self._conv3x3(up, "scratch.output_conv2.0", c0)
        ops.dpt_head_out(hidden.view(-1, hidden.shape[3]), self._conv_w("scratch.output_conv2.2", c2),
                         c2.bias.detach().float().contiguous(), self.activation, self.conf_activation,
                         preds.reshape(-1, preds.shape[-1]), conf.reshape(-1))
