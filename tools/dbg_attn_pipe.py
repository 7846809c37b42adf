"""Debug: the PIPE attention asm path against fp64 at small global lengths; prints the error per
head / d-block / q-block so a wrong fragment or stage shows where it lands."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "self-supervise-sfm_amd"))
from sailrecon_amd import ops  # noqa: E402

C, H, D = 1024, 16, 64
dev = "cuda"
for L in [int(x) for x in (sys.argv[1:] or ["256", "320", "512", "4096"])]:
    g = torch.Generator(device=dev).manual_seed(L)
    q = torch.randn(L, C, device=dev, generator=g).bfloat16()
    k = torch.randn(L, C, device=dev, generator=g).bfloat16() * 0.5
    v = torch.randn(L, C, device=dev, generator=g).bfloat16()
    o = torch.empty(L, C, device=dev, dtype=torch.bfloat16)
    kb = float(k.float().view(-1, H, D).norm(dim=-1).max())
    ops.attention(q, k, v, o, heads=H, head_dim=D, batch=1, lq=L, q_bstride=0, l0=L, k0_bstride=0, key_norm_max=kb)
    torch.cuda.synchronize()
    ref = torch.empty(L, C, dtype=torch.float64, device=dev)
    for h in range(H):
        c = slice(h * D, (h + 1) * D)
        s = (q[:, c].double() @ k[:, c].double().T) * D ** -0.5
        ref[:, c] = torch.softmax(s, -1) @ v[:, c].double()
    err = (o.double() - ref).abs()
    tot = float((o.double() - ref).norm() / ref.norm())
    print(f"L={L} rel {tot:.3e}")
    if tot > 1e-2:
        e = err.view(L, H, 2, 32)
        print("  max err per head:", [round(float(e[:, h].max()), 3) for h in range(H)])
        print("  per d-block:", [round(float(e[:, :, d].max()), 3) for d in range(2)])
        r = err.max(dim=1).values
        print("  per 32-row block (first 16):", [round(float(r[i * 32:(i + 1) * 32].max()), 3) for i in range(min(16, L // 32))])
        print("  per lane-half of d (cols 0-3,4-7 of 8):", [round(float(err.view(L, H, 8, 2, 4)[:, :, :, j].max()), 3) for j in range(2)])
