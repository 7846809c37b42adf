"""TEST-ONLY torch (CPU) implementation of the sailrecon_amd.ops API (= the C-ABI
semantics of include/sfm_amd.h), used to exercise the HOST orchestration of the
framework — row maps, subsample indices, token positions, frame sharding and the
RCCL/gloo collectives — on a machine without a GPU.

It is installed only by tests (``installed()`` context manager); the product path
never imports it and keeps failing loudly without libsfm_amd.so on a ROCm device.
"""

from __future__ import annotations

import contextlib
import math

import torch
import torch.nn.functional as F

from sailrecon_amd import _lib, ops as real_ops, runtime


def gemm(a, w, out, epi, *, bias=None, gamma=None, rows=None, qkv=None, patch=None, tag=None, q_scale=0.0,
         q_cols=0):
    M = a.shape[0] if rows is None else rows
    y = a[:M].float() @ w.float().t()
    if bias is not None:
        y = y + bias
    if qkv is not None and qkv.get("q_scale") and qkv.get("col_offset", 0) == 0:  # sr_gemm_epi.q_scale
        q_scale, q_cols = qkv["q_scale"], qkv["embed_dim"]
    if epi == _lib.SR_EPI_BIAS:
        if q_scale:
            y[:, :q_cols] *= q_scale
        out[:M] = y.to(out.dtype)
    elif epi == _lib.SR_EPI_BIAS_GELU:
        out[:M] = F.gelu(y).to(out.dtype)
    elif epi == _lib.SR_EPI_BIAS_RESID:
        out[:M] += y * gamma
    elif epi == _lib.SR_EPI_PATCH:
        sr, st, so = patch["seg_rows"], patch["seg_stride"], patch["seg_offset"]
        f = torch.arange(M) // sr
        p = torch.arange(M) % sr
        out[f * st + so + p] = y + patch["row_add"][p]
    elif epi == _lib.SR_EPI_QKV:
        C, D = qkv["embed_dim"], qkv.get("head_dim", 64)
        off = qkv.get("col_offset", 0)
        N = y.shape[1]
        cols = torch.arange(N) + off
        for h0 in range(0, N, D):
            region = int(cols[h0]) // C
            if region >= 2:
                continue
            seg = y[:, h0:h0 + D]
            nw = qkv.get("qn_w") if region == 0 else qkv.get("kn_w")
            nb = qkv.get("qn_b") if region == 0 else qkv.get("kn_b")
            if nw is not None:
                seg = F.layer_norm(seg, (D,), nw, nb, qkv.get("qk_eps", 1e-5))
            if qkv.get("rope_cos") is not None:
                py, px = _positions(qkv, M)
                cos, sin = qkv["rope_cos"], qkv["rope_sin"]
                q = D // 4

                def rot(v, pos):
                    c, s = cos[pos], sin[pos]
                    v1, v2 = v[:, :q], v[:, q:]
                    return torch.cat([v1 * c - v2 * s, v2 * c + v1 * s], 1)
                seg = torch.cat([rot(seg[:, :2 * q], py), rot(seg[:, 2 * q:], px)], 1)
            y[:, h0:h0 + D] = seg
        if q_scale:
            y[:, :q_cols] *= q_scale
        out[:M] = y.to(out.dtype)
    else:
        raise ValueError(epi)


def gemm_group(problems, epi, tag=None):
    for p in problems:
        gemm(p["a"], p["w"], p["out"], epi, bias=p.get("bias"), gamma=p.get("gamma"), qkv=p.get("qkv"),
             q_scale=p.get("q_scale", 0.0), q_cols=p.get("q_cols", 0))


def _positions(qkv, M):
    if qkv.get("pos_yx") is not None:
        p = qkv["pos_yx"].long()
        return p[:, 0], p[:, 1]
    rm = qkv.get("pos_rowmap")
    tr = rm.long()[:M] if rm is not None else qkv.get("pos_row_base", 0) + torch.arange(M)
    t = tr % qkv["tokens_per_frame"]
    ps, gw = qkv["patch_start"], qkv["grid_w"]
    p = (t - ps).clamp_min(0)
    special = t < ps
    py = torch.where(special, 0, p // gw + 1)
    px = torch.where(special, 0, p % gw + 1)
    return py, px


def attention(q, k0, v0, o, *, heads, head_dim, batch, lq, q_bstride, l0, k0_bstride, k1=None, v1=None, l1=0,
              k1_bstride=0, mask_mode=_lib.SR_MASK_NONE, n_anchor=0, scale=None, tag=None, lse=None,
              key_norm_max=0.0, mask=None, tail_readable=False, merge_o=None, merge_lse=None, sweep_stats=None,
              query_norm_max=0.0, q_scaled=False):
    """sr_attention's semantics (include/sfm_amd.h sr_attn_desc): the camera mask, SR_MASK_DENSE
    (nonzero = attend) / SR_MASK_ADD masks with zeros for a row without attended keys, and the
    merge-in of a disjoint key set's (merge_o, merge_lse).  sweep_stats (device diagnostics) is
    rejected: there is no sweep here.  ``q_scaled``: q holds c*q, c = scale*log2(e)."""
    if sweep_stats is not None:
        raise NotImplementedError("cpu_ops.attention: sweep_stats counts GPU waves")
    if mask_mode in (_lib.SR_MASK_DENSE, _lib.SR_MASK_ADD) and mask is None:
        raise ValueError("cpu_ops.attention: dense / additive mask_mode without a mask")
    D = head_dim
    scale = D ** -0.5 if scale is None else scale
    if q_scaled:  # (c q).k / log2(e) = scale q.k
        scale = 1.0 / math.log2(math.e)
    for b in range(batch):
        qs = q[b * q_bstride:b * q_bstride + lq].float()
        ks = [k0[b * k0_bstride:b * k0_bstride + l0].float()]
        vs = [v0[b * k0_bstride:b * k0_bstride + l0].float()]
        if l1 > 0:
            ks.append(k1[b * k1_bstride:b * k1_bstride + l1].float())
            vs.append(v1[b * k1_bstride:b * k1_bstride + l1].float())
        kk, vv = torch.cat(ks), torch.cat(vs)
        rows = slice(b * q_bstride, b * q_bstride + lq)
        for h in range(heads):
            sl = slice(h * D, (h + 1) * D)
            s = (qs[:, sl] @ kk[:, sl].t()) * scale
            if mask_mode == _lib.SR_MASK_CAMERA:
                i = torch.arange(lq)[:, None]
                j = torch.arange(kk.shape[0])[None]
                s = s.masked_fill(~((j < n_anchor) | (j == i)), float("-inf"))
            elif mask_mode == _lib.SR_MASK_DENSE:
                s = s.masked_fill(mask[b, h].to(torch.bool).logical_not(), float("-inf"))
            elif mask_mode == _lib.SR_MASK_ADD:
                s = s + mask[b, h].float()
            l2 = torch.logsumexp(s, -1) * (1.0 / math.log(2.0))
            p = torch.softmax(s, -1).nan_to_num(0.0)  # a row without attended keys: zeros (torch SDPA)
            y = p @ vv[:, sl]
            if merge_o is not None:  # sr_attn_merge's formula over the two disjoint key sets
                la = merge_lse[h, rows].float()
                m = torch.maximum(la, l2)
                wa, wb = torch.exp2(la - m), torch.exp2(l2 - m)
                tot = wa + wb
                y = (merge_o[rows, sl].float() * (wa / tot)[:, None] + y * (wb / tot)[:, None])
                l2 = m + torch.log2(tot)
            o[rows, sl] = y.to(o.dtype)
            if lse is not None:
                lse.view(batch, heads, lq)[b, h] = l2


def attn_merge(o_a, lse_a, o_b, lse_b, out, *, heads, head_dim, lse_out=None, tag=None):
    la, lb = lse_a.view(heads, -1).t(), lse_b.view(heads, -1).t()  # [rows, heads]
    m = torch.maximum(la, lb)
    wa, wb = torch.exp2(la - m), torch.exp2(lb - m)
    tot = wa + wb
    rows = out.shape[0]
    ya = o_a.float().view(rows, heads, head_dim) * (wa / tot)[..., None]
    yb = o_b.float().view(rows, heads, head_dim) * (wb / tot)[..., None]
    out.copy_((ya + yb).view(rows, heads * head_dim).to(out.dtype))
    if lse_out is not None:
        lse_out.view(heads, -1).copy_((m + torch.log2(tot)).t())


def attention_partials(q, k0, v0, o_parts, lse_parts, *, heads, head_dim, lq, l0, parts, scale=None, tag=None,
                       key_norm_max=0.0, tail_readable=False, query_norm_max=0.0, q_scaled=False):
    del tail_readable  # a memory-layout promise for the HIP sweep; no effect on the result
    assert l0 % parts == 0
    ch = l0 // parts
    for s in range(parts):
        attention(q, k0[s * ch:(s + 1) * ch], v0[s * ch:(s + 1) * ch], o_parts[s * lq:(s + 1) * lq], heads=heads,
                  head_dim=head_dim, batch=1, lq=lq, q_bstride=0, l0=ch, k0_bstride=0, scale=scale,
                  lse=lse_parts[s], q_scaled=q_scaled)


def attn_merge_n(o_parts, lse_parts, out, *, parts, rows, heads, head_dim, lse_out=None, seg_rows=None):
    blocks = []
    for p in range(parts):
        g = rows if seg_rows is None else seg_rows[p]
        lp = lse_parts.reshape(-1)[p * heads * rows:(p + 1) * heads * rows].view(rows // g, heads, g)
        blocks.append(lp.permute(0, 2, 1).reshape(rows, heads))
    ls = torch.stack(blocks)  # [parts, rows, heads]
    m = ls.max(0).values
    w = torch.exp2(ls - m)
    tot = w.sum(0)
    y = (o_parts[:parts * rows].float().view(parts, rows, heads, head_dim) * (w / tot)[..., None]).sum(0)
    out[:rows] = y.reshape(rows, heads * head_dim).to(out.dtype)
    if lse_out is not None:
        lse_out.view(heads, rows).copy_((m + torch.log2(tot)).t())


def layernorm(x, w, b, eps, out, rowmap=None, rows=None, x_copy=None):
    n = out.shape[0] if rows is None else rows
    src = x[rowmap.long()[:n]] if rowmap is not None else x[:n]
    if x_copy is not None:
        x_copy[:n] = src
    out[:n] = F.layer_norm(src, (x.shape[1],), w, b, eps).to(out.dtype)


def residual_layernorm(x, y, gamma, w, b, eps, out):
    x += (y.float() * (gamma if gamma is not None else 1.0))
    out.copy_(F.layer_norm(x, (x.shape[1],), w, b, eps).to(out.dtype))


def im2col_normalize(img, patch, out, kpad):
    mean = torch.tensor(real_ops._MEAN).view(1, 3, 1, 1)
    std = torch.tensor(real_ops._STD).view(1, 3, 1, 1)
    u = F.unfold((img - mean) / std, patch, stride=patch).transpose(1, 2).reshape(-1, 3 * patch * patch)
    out.zero_()
    out[:, :u.shape[1]] = u.to(out.dtype)


def set_special_tokens(x, frames, tokens_per_frame, table, type_of_frame):
    n = table.shape[1]
    xv = x.view(frames, tokens_per_frame, -1)
    xv[:, :n] = table[type_of_frame.reshape(-1).long()]


def copy_rows(dst, src, rows, rowmap=None):
    dst[:rows] = src[rowmap.long()[:rows]] if rowmap is not None else src[:rows]


def linear_small(a, w, bias, out, rows, act_in=0, lda=None):
    A = a.reshape(-1, w.shape[1])
    if lda == 0:
        A = A[:1].expand(rows, -1)
    A = A[:rows]
    if act_in:
        A = F.silu(A)
    out[:rows] = A @ w.t() + (bias if bias is not None else 0)


def silu(x, y):
    y.copy_(F.silu(x))


def adaln_modulate(xn, x, mod, out):
    sh, sc, g = mod.chunk(3, -1)
    out.copy_(g * (xn * (1 + sc) + sh) + x)


def pose_update(pred, delta, act, first):
    pred.copy_(delta if first else pred + delta)
    act.copy_(torch.cat([pred[:, :7], F.relu(pred[:, 7:])], -1))


def pose_decode(enc, hw, ext, intr):
    from oracle.sfm_oracle import pose_encoding_to_extri_intri
    e, i = pose_encoding_to_extri_intri(enc[None], hw)
    ext.copy_(e[0])
    intr.copy_(i[0])


_NAMES = ["gemm", "gemm_group", "attention", "attn_merge", "attention_partials", "attn_merge_n", "layernorm", "residual_layernorm",
          "im2col_normalize", "set_special_tokens", "copy_rows", "linear_small",
          "silu", "adaln_modulate", "pose_update", "pose_decode"]


@contextlib.contextmanager
def installed():
    """Route sailrecon_amd.ops through this module and allow CPU tensors."""
    saved = {n: getattr(real_ops, n) for n in _NAMES}
    saved_req = runtime.require_device
    g = globals()
    try:
        for n in _NAMES:
            setattr(real_ops, n, g[n])
        runtime.require_device = lambda t, who: None
        yield
    finally:
        for n, f in saved.items():
            setattr(real_ops, n, f)
        runtime.require_device = saved_req
