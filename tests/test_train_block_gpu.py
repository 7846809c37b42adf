"""Block forward-with-tape + backward (training engine) against torch autograd of the oracle's
fp32 Block (oracle.sfm_oracle.block = block.py:86-112) on the same parameters and input.

bf16 blocks (aggregator / DINO style, frame attention; qk-norm + 2-D RoPE or neither): bf16
GEMM / attention operands with fp32 accumulation against an fp32 reference -> 3e-2 rel-L2 on
the input grad and every parameter grad.  fp32 camera-trunk block (head_dim 128, camera mask,
f32 MFMA GEMMs, exact fp32 attention backward) -> 1e-4."""

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def _randomize(blk, seed):
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for n, p in blk.named_parameters():
            if n.endswith("gamma"):
                p.copy_(0.5 + torch.rand(p.shape, generator=g))
            elif "norm" in n and n.endswith("weight"):
                p.copy_(1 + 0.2 * torch.randn(p.shape, generator=g))
            elif n.endswith("bias"):
                p.copy_(0.1 * torch.randn(p.shape, generator=g))
            else:
                p.copy_(torch.randn(p.shape, generator=g) / p.shape[-1] ** 0.5)


def _positions(frames, P, gw):
    t = torch.arange(frames * P) % P
    p = (t - 5).clamp_min(0)
    return torch.stack([p // gw + 1, p % gw + 1], -1) * (t >= 5)[:, None]


@pytest.mark.parametrize("style", ["aggregator", "dino"])
def test_block_backward_bf16(style):
    from oracle import sfm_oracle as O
    from sailrecon_amd import runtime
    from sailrecon_amd.layers.block import Block
    from sailrecon_amd.layers.rope import RotaryPositionEmbedding2D
    from sailrecon_amd.train import engine
    from sailrecon_amd.train.params import FlatParams
    torch.manual_seed(0)
    C, H, frames, gh, gw = 256, 4, 3, 4, 5
    P = 5 + gh * gw
    R = frames * P
    agg = style == "aggregator"
    rope = RotaryPositionEmbedding2D(100) if agg else None
    blk = Block(dim=C, num_heads=H, init_values=0.01, qk_norm=agg, rope=rope)
    _randomize(blk, 1)
    sd = {k: v.detach().clone() for k, v in blk.state_dict().items()}
    blk = blk.to(DEV)
    fp = FlatParams(blk)
    blk.invalidate_packed()
    dt = torch.bfloat16
    pb = blk.packed(dt)
    qkv_epi = None
    if agg:
        tabs = rope.tables(C // H, max(gh, gw) + 1, DEV)
        qkv_epi = runtime.qkv_params(pb, tabs, pos_row_base=0, tokens_per_frame=P, patch_start=5, grid_w=gw)
    tape = engine.alloc_tape(R, C, 4 * C, dt, DEV, frames * H * P, separate_raw=qkv_epi is not None)
    fwd, bwd = engine.frame_attend_train(pb, frames, P)
    x = torch.randn(R, C)
    xd = x.to(DEV)
    engine.run_block_train(pb, xd, 0, R, tape, fwd, qkv_epi)
    dy = torch.randn(R, C)
    dx = dy.to(DEV)
    dxb = dx.bfloat16()
    fp.zero_grad()
    bp = engine.pack_bwd(blk, pb, dt)
    engine.block_bwd(pb, bp, engine.block_grads(blk), tape, dx, dxb, bwd, qkv_epi, engine.BwdScratch())
    torch.cuda.synchronize()

    # reference: autograd through the oracle block, fp32 CPU
    ref = {k: v.clone().requires_grad_(True) for k, v in sd.items() if v.is_floating_point()}
    xr = x.clone().requires_grad_(True)
    pos = _positions(frames, P, gw).view(frames, P, 2) if agg else None
    y = O.block(ref, "", xr.view(frames, P, C), H, 1e-5, pos=pos, qk_norm=agg,
                rope_base=100.0 if agg else None)
    y.backward(dy.view(frames, P, C))
    assert rel(xd, y.detach().reshape(R, C)) < 1e-2  # forward output
    assert rel(dx, xr.grad) < 3e-2, "input grad"
    for n, p in blk.named_parameters():
        assert rel(p.grad, ref[n].grad) < 3e-2, n


def test_block_backward_fp32_camera():
    from oracle import sfm_oracle as O
    from sailrecon_amd import _lib, ops
    from sailrecon_amd.layers.block import Block
    from sailrecon_amd.train import engine
    from sailrecon_amd.train.params import FlatParams
    torch.manual_seed(0)
    C, H, L, na = 256, 2, 24, 10   # head_dim 128 like the camera trunk
    blk = Block(dim=C, num_heads=H, init_values=0.01)
    _randomize(blk, 2)
    sd = {k: v.detach().clone() for k, v in blk.state_dict().items()}
    blk = blk.to(DEV)
    fp = FlatParams(blk)
    blk.invalidate_packed()
    dt = torch.float32
    pb = blk.packed(dt)
    tape = engine.alloc_tape(L, C, 4 * C, dt, DEV, 0, separate_raw=False)

    def fwd(qkv, o, lse):
        ops.attention(qkv[:, 0:C], qkv[:, C:2 * C], qkv[:, 2 * C:], o, heads=H, head_dim=C // H, batch=1, lq=L,
                      q_bstride=0, l0=L, k0_bstride=0, mask_mode=_lib.SR_MASK_CAMERA, n_anchor=na)

    def bwd(tp, dO, dqkv):
        q = tp.qkv
        ops.attention_bwd_small(q[:, 0:C], q[:, C:2 * C], q[:, 2 * C:], dO, dqkv[:, 0:C], dqkv[:, C:2 * C],
                                dqkv[:, 2 * C:], heads=H, head_dim=C // H, mask_mode=_lib.SR_MASK_CAMERA, n_anchor=na)
    x = torch.randn(L, C)
    xd = x.to(DEV)
    engine.run_block_train(pb, xd, 0, L, tape, fwd, None)
    dy = torch.randn(L, C)
    dx = dy.to(DEV)
    fp.zero_grad()
    bp = engine.pack_bwd(blk, pb, dt)
    engine.block_bwd(pb, bp, engine.block_grads(blk), tape, dx, None, bwd, None, engine.BwdScratch())
    torch.cuda.synchronize()
    ref = {k: v.clone().requires_grad_(True) for k, v in sd.items() if v.is_floating_point()}
    xr = x.clone().requires_grad_(True)
    allow = ~O.build_lr_mask(L, list(range(na)))
    y = O.block(ref, "", xr[None], H, 1e-5, mask=allow)
    y.backward(dy[None])
    assert rel(xd, y.detach()[0]) < 1e-5
    assert rel(dx, xr.grad) < 1e-4, "input grad"
    for n, p in blk.named_parameters():
        assert rel(p.grad, ref[n].grad) < 1e-4, n


def test_block_backward_fp32_qknorm_rope():
    """fp32 aggregator-style block (qk-norm + 2-D RoPE, autocast off): the backward runs
    sr_qk_bwd_f32 in place on dq|dk (VERDICT r3 missing 3) -> 1e-4 like the fp32 camera block."""
    from oracle import sfm_oracle as O
    from sailrecon_amd import ops, runtime
    from sailrecon_amd.layers.block import Block
    from sailrecon_amd.layers.rope import RotaryPositionEmbedding2D
    from sailrecon_amd.train import engine
    from sailrecon_amd.train.params import FlatParams
    torch.manual_seed(0)
    C, H, gh, gw = 256, 4, 4, 5
    P = 5 + gh * gw
    rope = RotaryPositionEmbedding2D(100)
    blk = Block(dim=C, num_heads=H, init_values=0.01, qk_norm=True, rope=rope)
    _randomize(blk, 3)
    sd = {k: v.detach().clone() for k, v in blk.state_dict().items()}
    blk = blk.to(DEV)
    fp = FlatParams(blk)
    blk.invalidate_packed()
    dt = torch.float32
    pb = blk.packed(dt)
    tabs = rope.tables(C // H, max(gh, gw) + 1, DEV)
    qkv_epi = runtime.qkv_params(pb, tabs, pos_row_base=0, tokens_per_frame=P, patch_start=5, grid_w=gw)
    tape = engine.alloc_tape(P, C, 4 * C, dt, DEV, 0, separate_raw=True)

    def fwd(qkv, o, lse):
        ops.attention(qkv[:, 0:C], qkv[:, C:2 * C], qkv[:, 2 * C:], o, heads=H, head_dim=C // H, batch=1, lq=P,
                      q_bstride=0, l0=P, k0_bstride=0)

    def bwd(tp, dO, dqkv):
        q = tp.qkv
        ops.attention_bwd_small(q[:, 0:C], q[:, C:2 * C], q[:, 2 * C:], dO, dqkv[:, 0:C], dqkv[:, C:2 * C],
                                dqkv[:, 2 * C:], heads=H, head_dim=C // H)
    x = torch.randn(P, C)
    xd = x.to(DEV)
    engine.run_block_train(pb, xd, 0, P, tape, fwd, qkv_epi)
    dy = torch.randn(P, C)
    dx = dy.to(DEV)
    fp.zero_grad()
    bp = engine.pack_bwd(blk, pb, dt)
    engine.block_bwd(pb, bp, engine.block_grads(blk), tape, dx, None, bwd, qkv_epi, engine.BwdScratch())
    torch.cuda.synchronize()
    ref = {k: v.clone().requires_grad_(True) for k, v in sd.items() if v.is_floating_point()}
    xr = x.clone().requires_grad_(True)
    pos = _positions(1, P, gw).view(1, P, 2)
    y = O.block(ref, "", xr[None], H, 1e-5, pos=pos, qk_norm=True, rope_base=100.0)
    y.backward(dy[None])
    assert rel(xd, y.detach()[0]) < 1e-5
    assert rel(dx, xr.grad) < 1e-4, "input grad"
    for n, p in blk.named_parameters():
        assert rel(p.grad, ref[n].grad) < 1e-4, n


def test_block_backward_c4_global():
    """BASELINE C4 (train_imc, 16 views): ONE full-width aggregator global block (C = 1024, 16
    heads, qk-norm + RoPE) forward-with-tape + backward over L_g = 16 x 1374 = 21,984 anchor
    tokens, the production attention shapes (frame_attend_train(pb, 1, L) is how train/model.py
    drives the global stack).  The upstream gradient is nonzero on 192 sampled output rows only,
    so the reference — autograd through the oracle's block (block.py:86-112, attention.py:70-122)
    in fp32 on the CPU — needs those rows' queries / MLP only, while every key / value row and so
    EVERY input row still receives a gradient through K and V.  Checked: the forward on the
    sampled rows, the input grad on the sampled rows and separately on 1024 other rows (their
    grad flows only through the attention backward's dK / dV), and every parameter grad; bf16
    operands vs the fp32 reference -> 3e-2 rel-L2 like the small bf16 block test."""
    from oracle import sfm_oracle as O
    import torch.nn.functional as F
    from sailrecon_amd import runtime
    from sailrecon_amd.layers.block import Block
    from sailrecon_amd.layers.rope import RotaryPositionEmbedding2D
    from sailrecon_amd.train import engine
    from sailrecon_amd.train.params import FlatParams
    torch.manual_seed(0)
    C, H, frames, gh, gw = 1024, 16, 16, 37, 37
    P = 5 + gh * gw
    L = frames * P
    D = C // H
    rope = RotaryPositionEmbedding2D(100)
    blk = Block(dim=C, num_heads=H, init_values=0.01, qk_norm=True, rope=rope)
    _randomize(blk, 4)
    sd = {k: v.detach().clone() for k, v in blk.state_dict().items()}
    blk = blk.to(DEV)
    fp = FlatParams(blk)
    blk.invalidate_packed()
    dt = torch.bfloat16
    pb = blk.packed(dt)
    tabs = rope.tables(D, max(gh, gw) + 1, DEV)
    qkv_epi = runtime.qkv_params(pb, tabs, pos_row_base=0, tokens_per_frame=P, patch_start=5, grid_w=gw)
    tape = engine.alloc_tape(L, C, 4 * C, dt, DEV, H * L, separate_raw=True)
    fwd, bwd = engine.frame_attend_train(pb, 1, L)
    x = torch.randn(L, C, generator=torch.Generator().manual_seed(5))
    xd = x.to(DEV)
    engine.run_block_train(pb, xd, 0, L, tape, fwd, qkv_epi)
    g = torch.Generator().manual_seed(6)
    rows = torch.sort(torch.randperm(L, generator=g)[:192]).values
    w = torch.randn(len(rows), C, generator=g)
    dy = torch.zeros(L, C)
    dy[rows] = w
    dx = dy.to(DEV)
    dxb = dx.bfloat16()
    fp.zero_grad()
    bp = engine.pack_bwd(blk, pb, dt)
    engine.block_bwd(pb, bp, engine.block_grads(blk), tape, dx, dxb, bwd, qkv_epi, engine.BwdScratch())
    torch.cuda.synchronize()

    # reference: the block's outputs at `rows` only, autograd through the oracle (fp32, CPU)
    ref = {k: v.clone().requires_grad_(True) for k, v in sd.items() if v.is_floating_point()}
    xr = x.clone().requires_grad_(True)
    pos = _positions(frames, P, gw)[None]                       # [1, L, 2]
    a = "attn."
    xn = O.layer_norm(xr, ref["norm1.weight"], ref["norm1.bias"], 1e-5)
    kv = F.linear(xn, ref[a + "qkv.weight"][C:], ref[a + "qkv.bias"][C:])       # K|V of every row
    qr = F.linear(xn[rows], ref[a + "qkv.weight"][:C], ref[a + "qkv.bias"][:C])  # Q of the sampled rows
    heads = lambda t: t.reshape(1, -1, H, D).transpose(1, 2)  # noqa: E731  [1, H, n, D]
    q = O.layer_norm(heads(qr), ref[a + "q_norm.weight"], ref[a + "q_norm.bias"], 1e-5)
    k = O.layer_norm(heads(kv[:, :C]), ref[a + "k_norm.weight"], ref[a + "k_norm.bias"], 1e-5)
    q = O.rope2d(q, pos[:, rows], 100.0)
    k = O.rope2d(k, pos, 100.0)
    o = F.scaled_dot_product_attention(q, k, heads(kv[:, C:]))
    o = o.transpose(1, 2).reshape(len(rows), C)
    x1 = xr[rows] + F.linear(o, ref[a + "proj.weight"], ref[a + "proj.bias"]) * ref["ls1.gamma"]
    y = x1 + O.mlp(ref, "mlp.", O.layer_norm(x1, ref["norm2.weight"], ref["norm2.bias"], 1e-5)) * ref["ls2.gamma"]
    (y * w).sum().backward()
    assert rel(xd[rows.to(DEV)], y.detach()) < 1e-2  # forward output
    others = torch.tensor(sorted(set(torch.randperm(L, generator=g)[:1100].tolist()) - set(rows.tolist()))[:1024])
    assert rel(dx[rows.to(DEV)], xr.grad[rows]) < 3e-2, "input grad (sampled rows)"
    assert float(xr.grad[others].norm()) > 0
    assert rel(dx[others.to(DEV)], xr.grad[others]) < 3e-2, "input grad through dK / dV"
    for n, p in blk.named_parameters():
        assert rel(p.grad, ref[n].grad) < 3e-2, n
