"""Attention backward (training step): sr_attention_bwd against torch
autograd of fp32 softmax attention on the same bf16-rounded q / k / v / dO, for the forward's
three key-segment shapes (frame: per-item keys; global: one item; global_reloc: a shared anchor
segment with batch stride 0 plus each item's own frame).  P and dS enter the MFMAs in bf16, as
in flash-attention backward: tolerance 2e-2 rel-L2."""

import math

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL = 2e-2


def _rel(a, b):
    return float((a - b).norm() / b.norm().clamp_min(1e-12))


def _ref(q, k, v, g, scale):
    q, k, v = (t.float().detach().requires_grad_(True) for t in (q, k, v))
    o = torch.softmax(q @ k.transpose(-1, -2) * scale, -1) @ v
    o.backward(g.float())
    return o.detach(), q.grad, k.grad, v.grad


@pytest.mark.parametrize("case", ["frame", "global", "reloc"])
@pytest.mark.parametrize("dt,D", [("bf16", 64), ("f32", 64), ("f32", 128)])
def test_attention_bwd_matches_autograd(case, dt, D):
    """bf16 operands: sr_attention_bwd at 2e-2.  fp32 operands (TrainGraph's fp32 mode):
    sr_attention_bwd_f32, exact fp32 against fp32 autograd at 2e-5 (head_dim 64 and 128)."""
    from sailrecon_amd import ops
    torch.manual_seed(0)
    H = 4
    C = H * D
    scale = D ** -0.5
    cast = (lambda t: t.bfloat16()) if dt == "bf16" else (lambda t: t)  # noqa: E731
    tol = TOL if dt == "bf16" else 2e-5
    if case == "frame":
        B, P = 3, 150
        x = cast(torch.randn(B * P, 3 * C, device=DEV))
        q, k, v = x[:, :C], x[:, C:2 * C], x[:, 2 * C:]
        kw = dict(batch=B, lq=P, q_bstride=P, l0=P, k0_bstride=P)
    elif case == "global":
        B, P = 1, 700
        x = cast(torch.randn(P, 3 * C, device=DEV))
        q, k, v = x[:, :C], x[:, C:2 * C], x[:, 2 * C:]
        kw = dict(batch=1, lq=P, q_bstride=P, l0=P, k0_bstride=P)
    else:
        B, P, A = 3, 150, 97
        x = cast(torch.randn(B * P, 3 * C, device=DEV))
        q, k, v = x[:, :C], x[:, C:2 * C], x[:, 2 * C:]
        ka = cast(torch.randn(A, 2 * C, device=DEV))
        k0, v0 = ka[:, :C], ka[:, C:]
        kw = dict(batch=B, lq=P, q_bstride=P, l0=A, k0_bstride=0, k1=k, v1=v, l1=P, k1_bstride=P)
    if case != "reloc":
        k0, v0 = k, v
    o = torch.empty(B * P, C, device=DEV, dtype=x.dtype)
    lse = torch.empty(B, H, P, device=DEV)
    ops.attention(q, k0, v0, o, heads=H, head_dim=D, lse=lse, **kw)
    g = cast(torch.randn(B * P, C, device=DEV))
    dq = torch.empty(B * P, C, device=DEV)
    dk0 = torch.empty(k0.shape[0], C, device=DEV)
    dv0 = torch.empty(k0.shape[0], C, device=DEV)
    dk1 = torch.empty(B * P, C, device=DEV) if case == "reloc" else None
    dv1 = torch.empty(B * P, C, device=DEV) if case == "reloc" else None
    delta = torch.empty(B, H, P, device=DEV)
    ops.attention_bwd(q, k0, v0, o, lse, g, dq, dk0, dv0, delta, heads=H, dk1=dk1, dv1=dv1, **kw)
    torch.cuda.synchronize()
    # reference, per item and head
    def heads_of(t, rows):
        return t.reshape(rows, H, D).transpose(0, 1)
    dq_r = torch.zeros(B * P, C, device=DEV)
    dk0_r = torch.zeros_like(dk0)
    dv0_r = torch.zeros_like(dv0)
    dk1_r = torch.zeros(B * P, C, device=DEV)
    dv1_r = torch.zeros(B * P, C, device=DEV)
    for b in range(B):
        rs = slice(b * P, (b + 1) * P)
        qb, gb = heads_of(q[rs], P), heads_of(g[rs], P)
        if case == "frame":
            kk, vv = heads_of(k[rs], P), heads_of(v[rs], P)
        elif case == "global":
            kk, vv = heads_of(k, P), heads_of(v, P)
        else:
            kk = torch.cat([heads_of(k0, A), heads_of(k[rs], P)], 1)
            vv = torch.cat([heads_of(v0, A), heads_of(v[rs], P)], 1)
        o_r, dqh, dkh, dvh = _ref(qb, kk, vv, gb, scale)
        assert _rel(heads_of(o[rs], P).float(), o_r) < tol
        dq_r[rs] = dqh.transpose(0, 1).reshape(P, C)
        if case == "reloc":
            dk0_r += dkh[:, :A].transpose(0, 1).reshape(A, C)
            dv0_r += dvh[:, :A].transpose(0, 1).reshape(A, C)
            dk1_r[rs] = dkh[:, A:].transpose(0, 1).reshape(P, C)
            dv1_r[rs] = dvh[:, A:].transpose(0, 1).reshape(P, C)
        elif case == "frame":
            dk0_r[rs] = dkh.transpose(0, 1).reshape(P, C)
            dv0_r[rs] = dvh.transpose(0, 1).reshape(P, C)
        else:
            dk0_r[:] = dkh.transpose(0, 1).reshape(P, C)
            dv0_r[:] = dvh.transpose(0, 1).reshape(P, C)
        # lse (log2 domain) of this item's rows
        s = (qb.float() @ kk.float().transpose(-1, -2)) * scale
        assert torch.allclose(lse[b], torch.logsumexp(s, -1) / math.log(2), rtol=0, atol=2e-2 if dt == "bf16" else 1e-4)
    assert _rel(dq, dq_r) < tol
    assert _rel(dk0, dk0_r) < tol and _rel(dv0, dv0_r) < tol
    if case == "reloc":
        assert _rel(dk1, dk1_r) < tol and _rel(dv1, dv1_r) < tol


@pytest.mark.parametrize("case,P", [("frame", 1374), ("frame", 256), ("frame", 337), ("frame", 384), ("frame", 511),
                                    ("frame", 512), ("frame", 200), ("global", 1100), ("reloc", 300),
                                    ("anchor", 150)])
def test_attention_bwd_pipe(case, P):
    """SR_ATTN_BWD_PIPE / SR_ATTN_BWD_DQ_PIPE: the hand-scheduled dK/dV and dQ sweeps
    (tools/gen_attn_bwd_pipe.py) give bit-identical dQ / dK / dV to the compiled sweeps: full tile
    counts 4..21 (every remainder of the asm's 4-tile loop), ragged last tiles (17, 30, 44, 60, 63
    rows) and none, fewer than 4 full tiles (P = 200: the compiled sweeps run), keys shared across
    the batch (reloc: two key segments, dQ compiled, dK/dV segment 1 per item in the asm; anchor:
    one shared segment of 700 keys, dQ in the asm for 150 queries per item, dK/dV compiled)."""
    from sailrecon_amd import ops
    torch.manual_seed(2)
    H, D = 4, 64
    C = H * D
    if case == "frame":
        B, A = 3, 0
        kw = dict(batch=B, lq=P, q_bstride=P, l0=P, k0_bstride=P)
    elif case == "global":
        B, A = 1, 0
        kw = dict(batch=1, lq=P, q_bstride=P, l0=P, k0_bstride=P)
    elif case == "anchor":
        B, A = 3, 700
        kw = dict(batch=B, lq=P, q_bstride=P, l0=A, k0_bstride=0)
    else:
        B, A = 3, 301
        kw = dict(batch=B, lq=P, q_bstride=P, l0=A, k0_bstride=0, l1=P, k1_bstride=P)
    x = torch.randn(B * P, 3 * C, device=DEV).bfloat16()
    q, k, v = x[:, :C], x[:, C:2 * C], x[:, 2 * C:]
    if case in ("reloc", "anchor"):
        ka = torch.randn(A, 2 * C, device=DEV).bfloat16()
        k0, v0 = ka[:, :C], ka[:, C:]
        if case == "reloc":
            kw.update(k1=k, v1=v)
    else:
        k0, v0 = k, v
    o = torch.empty(B * P, C, device=DEV, dtype=torch.bfloat16)
    lse = torch.empty(B, H, P, device=DEV)
    ops.attention(q, k0, v0, o, heads=H, head_dim=D, lse=lse, **kw)
    g = torch.randn(B * P, C, device=DEV).bfloat16()
    outs = []
    for pipe in (0, 1):
        dq = torch.full((B * P, C), float("nan"), device=DEV)
        dk0 = torch.full((k0.shape[0], C), float("nan"), device=DEV)
        dv0 = torch.full((k0.shape[0], C), float("nan"), device=DEV)
        dk1 = torch.full((B * P, C), float("nan"), device=DEV) if case == "reloc" else None
        dv1 = torch.full((B * P, C), float("nan"), device=DEV) if case == "reloc" else None
        delta = torch.empty(B, H, P, device=DEV)
        with ops.tuning(SR_ATTN_BWD_PIPE=pipe, SR_ATTN_BWD_DQ_PIPE=2 * pipe, SR_ATTN_BWD_CAT=0):
            ops.attention_bwd(q, k0, v0, o, lse, g, dq, dk0, dv0, delta, heads=H, dk1=dk1, dv1=dv1, **kw)
            asm_dkdv = pipe and P >= 256 and case not in ("reloc", "anchor")
            want = "attn_bwd_dkdv_pipe_kernel<0>" if asm_dkdv else "attn_bwd_dkdv_kernel<0>"
            assert ops.last_kernel() == want
        outs.append([t for t in (dq, dk0, dv0, dk1, dv1) if t is not None])
    torch.cuda.synchronize()
    for a, b in zip(*outs):
        assert torch.isfinite(a).all()
        assert torch.equal(a, b)


@pytest.mark.parametrize("B,P", [(3, 300), (2, 1374), (5, 64)])
def test_attention_bwd_concatenated_items(B, P):
    """SR_ATTN_BWD_CAT: anchors shared by a batch whose queries are consecutive rows run as ONE
    asm dK/dV sweep over the concatenated queries (tiles straddling items; each row's lse / -delta
    found per tile).  Equal to the compiled per-item sweep up to fp32 summation grouping, and
    deterministic; dQ and the per-item segment are unchanged."""
    from sailrecon_amd import ops
    torch.manual_seed(4)
    H, D, A = 4, 64, 301
    C = H * D
    kw = dict(batch=B, lq=P, q_bstride=P, l0=A, k0_bstride=0, l1=P, k1_bstride=P)
    x = torch.randn(B * P, 3 * C, device=DEV).bfloat16()
    q, k, v = x[:, :C], x[:, C:2 * C], x[:, 2 * C:]
    ka = torch.randn(A, 2 * C, device=DEV).bfloat16()
    k0, v0 = ka[:, :C], ka[:, C:]
    kw.update(k1=k, v1=v)
    o = torch.empty(B * P, C, device=DEV, dtype=torch.bfloat16)
    lse = torch.empty(B, H, P, device=DEV)
    ops.attention(q, k0, v0, o, heads=H, head_dim=D, lse=lse, **kw)
    g = torch.randn(B * P, C, device=DEV).bfloat16()
    outs = []
    for cat in (0, 1, 1):
        dq = torch.empty(B * P, C, device=DEV)
        dk0 = torch.full((A, C), float("nan"), device=DEV)
        dv0 = torch.full((A, C), float("nan"), device=DEV)
        dk1, dv1 = torch.empty(B * P, C, device=DEV), torch.empty(B * P, C, device=DEV)
        delta = torch.empty(B, H, P, device=DEV)
        with ops.tuning(SR_ATTN_BWD_CAT=cat):
            ops.attention_bwd(q, k0, v0, o, lse, g, dq, dk0, dv0, delta, heads=H, dk1=dk1, dv1=dv1, **kw)
            want = "attn_bwd_dkdv_pipe_kernel<0, cat>" if cat and B * P >= 256 else "attn_bwd_dkdv_kernel<0>"
            assert ops.last_kernel() == want
        outs.append((dq, dk0, dv0, dk1, dv1))
    torch.cuda.synchronize()
    for i, (a, b, c) in enumerate(zip(*outs)):
        assert torch.isfinite(b).all()
        assert torch.equal(b, c)  # deterministic
        if i in (1, 2):  # dK / dV of the shared anchors: summation grouping only
            err = float((a - b).abs().max() / a.abs().max())
            print(f"B={B} P={P} {'dk0' if i == 1 else 'dv0'} concatenated vs per-item: {err:.2e}")
            assert err <= 1e-5
        else:
            assert torch.equal(a, b)
