"""PatchEmbed mirror (reference: sailrecon/layers/patch_embed.py:25-84).

Inside the aggregator the 14x14/stride-14 conv runs as im2col (sr_im2col_normalize, fused
with the image normalisation) + GEMM with the SR_EPI_PATCH epilogue (bias + positional add +
token-row remap).  A standalone ``PatchEmbed.forward(x)`` (patch_embed.py:67-84) is the same
im2col without normalisation + a bias-epilogue GEMM: [B, 3, H, W] -> [B, HW, C] (or
[B, H', W', C] without ``flatten_embedding``), bf16 under autocast, exact fp32 otherwise.
"""

import torch
from torch import Tensor, nn

from .. import _lib, ops, runtime


def make_2tuple(x):
    if isinstance(x, tuple):
        assert len(x) == 2
        return x
    assert isinstance(x, int)
    return (x, x)


class PatchEmbed(nn.Module):
    def __init__(self, img_size=224, patch_size=16, in_chans=3, embed_dim=768, norm_layer=None,
                 flatten_embedding=True) -> None:
        super().__init__()
        image_hw = make_2tuple(img_size)
        patch_hw = make_2tuple(patch_size)
        self.img_size = image_hw
        self.patch_size = patch_hw
        self.patches_resolution = (image_hw[0] // patch_hw[0], image_hw[1] // patch_hw[1])
        self.num_patches = self.patches_resolution[0] * self.patches_resolution[1]
        self.in_chans = in_chans
        self.embed_dim = embed_dim
        self.flatten_embedding = flatten_embedding
        self.proj = nn.Conv2d(in_chans, embed_dim, kernel_size=patch_hw, stride=patch_hw)
        self.norm = norm_layer(embed_dim) if norm_layer else nn.Identity()

    def forward(self, x: Tensor) -> Tensor:
        runtime.require_device(x, "PatchEmbed")
        _, _, H, W = x.shape
        ph, pw = self.patch_size
        assert H % ph == 0, f"Input image height {H} is not a multiple of patch height {ph}"
        assert W % pw == 0, f"Input image width {W} is not a multiple of patch width: {pw}"
        if ph != pw or self.in_chans != 3:
            raise NotImplementedError("PatchEmbed.forward: square patches over 3 channels")
        if not isinstance(self.norm, nn.Identity):
            raise NotImplementedError("PatchEmbed.forward: norm_layer (unused by every SailRecon config)")
        dtype = runtime.compute_dtype()
        B = x.shape[0]
        C = self.embed_dim
        kt = 64 if dtype == torch.bfloat16 else 32
        kpad = -(-3 * ph * pw // kt) * kt
        gh, gw = H // ph, W // pw
        cols = torch.empty(B * gh * gw, kpad, device=x.device, dtype=dtype)
        ops.im2col_normalize(x.detach().float().contiguous(), ph, cols, kpad, normalize=False)
        w = torch.zeros(C, kpad, device=x.device, dtype=dtype)
        w[:, : 3 * ph * pw] = self.proj.weight.detach().reshape(C, -1).to(dtype)
        out = torch.empty(B * gh * gw, C, device=x.device, dtype=dtype)
        bias = None if self.proj.bias is None else self.proj.bias.detach().float().contiguous()
        ops.gemm(cols, w, out, _lib.SR_EPI_BIAS, bias=bias)
        if not self.flatten_embedding:
            return out.view(B, gh, gw, C)
        return out.view(B, gh * gw, C)
