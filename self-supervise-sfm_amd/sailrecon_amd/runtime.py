"""Block executor: packed weights + workspace + the per-block kernel sequence.

One transformer Block (reference block.py:86-112, attention.py:70-122,
mlp.py:34-40) is seven launches on the HIP path:

    LN1 -> GEMM qkv (+bias, qk-LayerNorm, RoPE fused) -> attention
        -> GEMM proj (+bias, LayerScale, residual add fused, in place on x)
    LN2 -> GEMM fc1 (+bias, erf-GELU fused) -> GEMM fc2 (+bias, LayerScale, residual)

The residual stream x is fp32 [rows, C] (as under the reference's bf16 autocast,
where LayerScale's fp32 gamma promotes every residual add to fp32).  Workspace
buffers are indexed with the SAME absolute rows as x, so blocks over disjoint row
ranges (global anchors vs reloc queries) never share scratch.
"""

from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Callable, Dict, Optional, Tuple

import torch

from . import _lib, ops

Tensor = torch.Tensor


def require_device(t: Tensor, who: str) -> None:
    """The product path runs only through libsfm_amd.so on a ROCm device: fail loudly."""
    if not t.is_cuda:
        raise RuntimeError(f"sailrecon_amd {who} runs on the HIP path only (tensors must be on a ROCm device)")


def to_device(t: Tensor, device) -> Tensor:
    """Small host->device copy (pinned, async) for index tables."""
    if torch.device(device).type == "cuda":
        return t.pin_memory().to(device, non_blocking=True)
    return t.to(device)


def compute_dtype(explicit: Optional[torch.dtype] = None) -> torch.dtype:
    """bf16 when the caller runs under autocast (demo_imc_forward.py:93), else fp32 parity mode."""
    if explicit is not None:
        return torch.bfloat16 if explicit in (torch.bfloat16, torch.float16) else torch.float32
    if torch.is_autocast_enabled("cuda"):
        return torch.bfloat16
    return torch.float32


@dataclass
class PackedBlock:
    dim: int
    heads: int
    head_dim: int
    eps: float
    qk_eps: float
    qk_norm: bool
    ln1_w: Tensor
    ln1_b: Tensor
    ln2_w: Tensor
    ln2_b: Tensor
    w_qkv: Tensor
    b_qkv: Optional[Tensor]
    qn_w: Optional[Tensor]
    qn_b: Optional[Tensor]
    kn_w: Optional[Tensor]
    kn_b: Optional[Tensor]
    w_proj: Tensor
    b_proj: Optional[Tensor]
    g1: Tensor
    w_fc1: Tensor
    b_fc1: Optional[Tensor]
    w_fc2: Tensor
    b_fc2: Optional[Tensor]
    g2: Tensor
    k_bound: float = -1.0  # key_norm_bound cache (-1: not computed yet)
    q_bound: float = -1.0  # query_norm_bound cache


def key_norm_bound(pb: PackedBlock) -> float:
    """Static bound of every key's per-head 2-norm for a qk-norm block (attention.py:49-50,78):
    k = LN(x) * w + b with |LN(x)| <= sqrt(head_dim), then RoPE (a rotation), so
    |k| <= sqrt(head_dim) max|w| + |b|; x (1 + 2^-6) covers the bf16 rounding of k.  0 without
    qk-norm (the attention then scans the keys).  One host read per packing, cached."""
    if pb.k_bound < 0.0:
        if not pb.qk_norm or pb.kn_w is None:
            pb.k_bound = 0.0
        else:
            w = float(pb.kn_w.abs().max())
            b = float(pb.kn_b.norm()) if pb.kn_b is not None else 0.0
            pb.k_bound = (pb.head_dim ** 0.5 * w + b) * (1.0 + 2.0 ** -6)
    return pb.k_bound


def query_norm_bound(pb: PackedBlock) -> float:
    """key_norm_bound's bound for the queries (q_norm, attention.py:49-50,77): with it the
    attention sees the static score bound scale * |q| * |k| and computes the per-dimension key box
    (ops.attention's query_norm_max) only when that bound leaves the fixed-offset window."""
    if pb.q_bound < 0.0:
        if not pb.qk_norm or pb.qn_w is None:
            pb.q_bound = 0.0
        else:
            w = float(pb.qn_w.abs().max())
            b = float(pb.qn_b.norm()) if pb.qn_b is not None else 0.0
            pb.q_bound = (pb.head_dim ** 0.5 * w + b) * (1.0 + 2.0 ** -6)
    return pb.q_bound


def _f32(t: Optional[Tensor]) -> Optional[Tensor]:
    return None if t is None else t.detach().float().contiguous()


def _gamma(ls, dim: int, ref: Tensor) -> Tensor:
    g = getattr(ls, "gamma", None)
    return _f32(g) if g is not None else torch.ones(dim, device=ref.device, dtype=torch.float32)


def pack_block(blk, dtype: torch.dtype) -> PackedBlock:
    a = blk.attn
    w = lambda t: t.detach().to(dtype).contiguous()  # noqa: E731
    qk = bool(getattr(a, "qk_norm", False))
    return PackedBlock(
        dim=a.qkv.in_features, heads=a.num_heads, head_dim=a.head_dim, eps=blk.norm1.eps,
        qk_eps=a.q_norm.eps if qk else 1e-5, qk_norm=qk,
        ln1_w=_f32(blk.norm1.weight), ln1_b=_f32(blk.norm1.bias),
        ln2_w=_f32(blk.norm2.weight), ln2_b=_f32(blk.norm2.bias),
        w_qkv=w(a.qkv.weight), b_qkv=_f32(a.qkv.bias),
        qn_w=_f32(a.q_norm.weight) if qk else None, qn_b=_f32(a.q_norm.bias) if qk else None,
        kn_w=_f32(a.k_norm.weight) if qk else None, kn_b=_f32(a.k_norm.bias) if qk else None,
        w_proj=w(a.proj.weight), b_proj=_f32(a.proj.bias), g1=_gamma(blk.ls1, a.qkv.in_features, a.qkv.weight),
        w_fc1=w(blk.mlp.fc1.weight), b_fc1=_f32(blk.mlp.fc1.bias),
        w_fc2=w(blk.mlp.fc2.weight), b_fc2=_f32(blk.mlp.fc2.bias),
        g2=_gamma(blk.ls2, a.qkv.in_features, a.qkv.weight),
    )


def pack_attention(a, dtype: torch.dtype) -> PackedBlock:
    """The attention half of pack_block for a standalone ``Attention.forward``."""
    w = lambda t: t.detach().to(dtype).contiguous()  # noqa: E731
    qk = bool(getattr(a, "qk_norm", False))
    dim = a.qkv.in_features
    return PackedBlock(
        dim=dim, heads=a.num_heads, head_dim=a.head_dim, eps=0.0, qk_eps=a.q_norm.eps if qk else 1e-5, qk_norm=qk,
        ln1_w=None, ln1_b=None, ln2_w=None, ln2_b=None, w_qkv=w(a.qkv.weight), b_qkv=_f32(a.qkv.bias),
        qn_w=_f32(a.q_norm.weight) if qk else None, qn_b=_f32(a.q_norm.bias) if qk else None,
        kn_w=_f32(a.k_norm.weight) if qk else None, kn_b=_f32(a.k_norm.bias) if qk else None,
        w_proj=w(a.proj.weight), b_proj=_f32(a.proj.bias), g1=None, w_fc1=None, b_fc1=None, w_fc2=None, b_fc2=None,
        g2=None)


class Workspace:
    """Grow-only device scratch, keyed by name (reused across forwards).  Buffers are zeroed when
    allocated and carry PAD_ROWS rows of padding, so every row past a view's end is readable and
    finite (ops.attention(tail_readable=True): the hand-scheduled attention sweep stages a ragged
    last key tile whole)."""

    PAD_ROWS = 64

    def __init__(self):
        self._bufs: Dict[str, Tensor] = {}

    def get(self, name: str, rows: int, cols: int, dtype: torch.dtype, device) -> Tensor:
        t = self._bufs.get(name)
        need = rows * cols
        if t is None or t.dtype != dtype or t.device != torch.device(device) or \
                t.numel() < need + self.PAD_ROWS * cols:
            t = torch.zeros(need + self.PAD_ROWS * max(cols, 1), dtype=dtype, device=device)
            self._bufs[name] = t
        return t[:need].view(rows, cols)

    def clear(self):
        self._bufs.clear()


@dataclass
class BlockScratch:
    xn: Tensor   # [R, C] dtype
    qkv: Tensor  # [R, 3C] dtype
    o: Tensor    # [R, C] dtype
    h: Tensor    # [R, 4C] dtype


def scratch(ws: Workspace, rows: int, dim: int, hidden: int, dtype: torch.dtype, device, tag: str = "") -> BlockScratch:
    return BlockScratch(xn=ws.get("xn" + tag, rows, dim, dtype, device),
                        qkv=ws.get("qkv" + tag, rows, 3 * dim, dtype, device),
                        o=ws.get("o" + tag, rows, dim, dtype, device),
                        h=ws.get("h" + tag, rows, hidden, dtype, device))


# The attention's c*q (c = scale * log2(e): scores in the exp2 domain) is formed by the QKV GEMM's
# epilogue from its fp32 value and rounded to bf16 ONCE (sr_gemm_epi.q_scale), and the attention
# takes it as is (sr_attn_desc.q_scaled).  The reference rounds q once (autocast SDPA input,
# attention.py:103-109) and scales inside SDPA; forming c * bf16(q) in the kernel instead rounded q
# twice.  Forward-only (inference) convention: the training tape keeps plain q
# for sr_attention_bwd.  SR_Q_PRESCALE=0 restores the in-kernel product (A/B).
_Q_PRESCALE = os.environ.get("SR_Q_PRESCALE", "1") != "0"
_LOG2E = 1.4426950408889634


def q_prescale(pb: PackedBlock) -> float:
    """c = head_dim^-0.5 * log2(e) for a bf16 pack (0.0: fp32 parity mode keeps plain q)."""
    if not _Q_PRESCALE or pb.w_qkv.dtype != torch.bfloat16 or pb.head_dim != 64:
        return 0.0
    return pb.head_dim ** -0.5 * _LOG2E


def qkv_params(pb: PackedBlock, rope: Optional[Tuple[Tensor, Tensor]], prescale: bool = False,
               **pos) -> Optional[dict]:
    """Epilogue parameters for the fused qkv GEMM; None if plain bias suffices.  ``prescale``: the
    Q block leaves as c*q (q_prescale; the attention then takes q_scaled=True)."""
    if not pb.qk_norm and rope is None:
        return None
    d = dict(embed_dim=pb.dim, head_dim=pb.head_dim, qk_eps=pb.qk_eps,
             qn_w=pb.qn_w, qn_b=pb.qn_b, kn_w=pb.kn_w, kn_b=pb.kn_b)
    if prescale and q_prescale(pb):
        d["q_scale"] = q_prescale(pb)
    if rope is not None:
        d["rope_cos"], d["rope_sin"] = rope
        d.update(pos)
    return d


def qkv_gemm(pb: PackedBlock, xn: Tensor, w: Tensor, out: Tensor, bias, qkv_epi: Optional[dict],
             q_scale: float = 0.0) -> None:
    """The QKV projection: the fused qk-norm / RoPE epilogue when ``qkv_epi`` is set, else plain bias
    (DINO), whose Q block (the first pb.dim output columns) leaves scaled by ``q_scale`` if nonzero."""
    if qkv_epi is None:
        ops.gemm(xn, w, out, _lib.SR_EPI_BIAS, bias=bias, tag="gemm", q_scale=q_scale,
                 q_cols=pb.dim if q_scale else 0)
    else:
        ops.gemm(xn, w, out, _lib.SR_EPI_QKV, bias=bias, qkv=qkv_epi, tag="gemm")


# Residual updates folded into the next LayerNorm.  The reference's autocast
# Linear returns bf16 and LayerScale / the residual add happen outside it (block.py:86-112,
# layer_scale.py:22-23); so the proj / fc2 GEMMs may end in the plain bias epilogue (their output
# in the compute dtype, as the reference has it) and x += gamma * y streams through
# sr_residual_layernorm together with the LayerNorm that reads x next:
#   SR_FUSED_RESID_LN=1: proj -> LN2 of the same block;
#   SR_DEFER_RESID=1:    fc2 -> LN1 of the next block over the same rows (DINO block i -> i+1; the
#                        global / reloc blocks of layer l -> the frame block of layer l+1), where no
#                        other reader of x comes in between (Pending / run_block's ``pending``).
# Measured (round 3, proj only): the GEMMs' MFMA utilisation 0.378 -> 0.391 at C3 and the step even
# (409.9 / 409.9 vs 409.1 / 408.6 ms): the fused pass moves 12 B per element where LayerNorm moves 6.
# Round 6, one box, interleaved, 2 runs each (profiles/r06_j13_bench_rm*.log; proj-fused, fc2-deferred):
#   neither 80.55 / 80.67 views/s (gemm_mfma_util 0.391 / 0.392), proj 80.15 / 80.31 (0.402 / 0.404),
#   fc2 80.63 / 80.63 (0.401 / 0.401), both 80.13 / 80.03 (0.411 / 0.411): the fc2 deferral is the
#   default -- level on the step, and the reference's order (bf16 Linear output, then LayerScale and
#   the fp32 residual add outside it)
_FUSED_RESID_LN = os.environ.get("SR_FUSED_RESID_LN", "0") == "1"
_DEFER_RESID = os.environ.get("SR_DEFER_RESID", "1") == "1"


@dataclass
class Pending:
    """A residual update x[r0:r1] += gamma * y deferred to the next LayerNorm over those rows
    (y [r1 - r0, C] in the compute dtype: a GEMM's bias-epilogue output)."""
    r0: int
    r1: int
    y: Tensor
    gamma: Tensor


def defer_enabled(pb: PackedBlock) -> bool:
    return _DEFER_RESID and pb.w_fc2 is not None and pb.w_fc2.shape[0] in ops.RESIDUAL_LN_COLS


def layernorm_pending(x: Tensor, r0: int, r1: int, w, b, eps: float, xn: Tensor, pending) -> None:
    """xn = LN(x[r0:r1]) after applying the ``pending`` residual updates that cover these rows
    (each one exactly once: applied updates are removed from the list)."""
    if not pending:
        ops.layernorm(x[r0:r1], w, b, eps, xn)
        return
    cur = r0
    for p in sorted([p for p in pending if p.r0 < r1 and p.r1 > r0], key=lambda p: p.r0):
        if p.r0 < r0 or p.r1 > r1:
            raise RuntimeError("a pending residual update straddles the LayerNorm's rows")
        if cur < p.r0:
            ops.layernorm(x[cur:p.r0], w, b, eps, xn[cur - r0:p.r0 - r0])
        ops.residual_layernorm(x[p.r0:p.r1], p.y, p.gamma, w, b, eps, xn[p.r0 - r0:p.r1 - r0])
        pending.remove(p)
        cur = p.r1
    if cur < r1:
        ops.layernorm(x[cur:r1], w, b, eps, xn[cur - r0:])


def proj_residual_ln2(pb: PackedBlock, xs: Tensor, o: Tensor, qkv: Tensor, xn: Tensor) -> None:
    """xs += g1 * proj(o); xn = norm2(xs) (block.py:86-89).  Default: the projection GEMM's fp32
    bias*gamma + residual epilogue, then LayerNorm.  SR_FUSED_RESID_LN=1: the GEMM writes its bias
    output in the compute dtype into the dead q slot of ``qkv`` and sr_residual_layernorm streams
    the residual update and LN2 in one pass."""
    C = pb.w_proj.shape[0]
    if _FUSED_RESID_LN and C in ops.RESIDUAL_LN_COLS and qkv.shape[1] >= C:
        y = qkv[:, :C]
        ops.gemm(o, pb.w_proj, y, _lib.SR_EPI_BIAS, bias=pb.b_proj, tag="gemm")
        ops.residual_layernorm(xs, y, pb.g1, pb.ln2_w, pb.ln2_b, pb.eps, xn)
    else:
        ops.gemm(o, pb.w_proj, xs, _lib.SR_EPI_BIAS_RESID, bias=pb.b_proj, gamma=pb.g1, tag="gemm")
        ops.layernorm(xs, pb.ln2_w, pb.ln2_b, pb.eps, xn)


def mlp_residual(pb: PackedBlock, x: Tensor, r0: int, r1: int, sc: BlockScratch, defer: bool) -> Optional[Pending]:
    """fc1 (+GELU) and fc2 with the LayerScale residual: x[r0:r1] += g2 * fc2(gelu(fc1(xn))).
    ``defer``: fc2 ends in the bias epilogue into the block's dead attention-output rows sc.o and
    the update is returned as a Pending for the next LayerNorm over these rows."""
    xs, xn, h, o = x[r0:r1], sc.xn[r0:r1], sc.h[r0:r1], sc.o[r0:r1]
    hid = pb.w_fc1.shape[0]
    ops.gemm(xn, pb.w_fc1, h[:, :hid], _lib.SR_EPI_BIAS_GELU, bias=pb.b_fc1, tag="gemm")
    if defer and defer_enabled(pb) and o.shape[1] >= pb.w_fc2.shape[0]:
        y = o[:, :pb.w_fc2.shape[0]]
        ops.gemm(h[:, :hid], pb.w_fc2, y, _lib.SR_EPI_BIAS, bias=pb.b_fc2, tag="gemm")
        return Pending(r0, r1, y, pb.g2)
    ops.gemm(h[:, :hid], pb.w_fc2, xs, _lib.SR_EPI_BIAS_RESID, bias=pb.b_fc2, gamma=pb.g2, tag="gemm")
    return None


def run_block(pb: PackedBlock, x: Tensor, r0: int, r1: int, sc: BlockScratch,
              attend: Callable[[Tensor, Tensor], None], qkv_epi: Optional[dict], tag: str = "blk",
              pending: Optional[list] = None, defer: bool = False, q_scale: float = 0.0) -> Optional[Pending]:
    """x[r0:r1] <- Block(x[r0:r1]); ``attend(qkv_rows, o_rows)`` launches the attention.
    ``pending``: deferred residual updates of earlier blocks, applied by this block's LN1 (the list
    is consumed).  ``defer``: leave this block's fc2 residual pending (returned; see mlp_residual).
    ``q_scale``: the plain-bias QKV projection's Q block leaves scaled (qkv_gemm; a fused epilogue
    carries its own in ``qkv_epi``)."""
    xs = x[r0:r1]
    xn, qkv, o = sc.xn[r0:r1], sc.qkv[r0:r1], sc.o[r0:r1]
    layernorm_pending(x, r0, r1, pb.ln1_w, pb.ln1_b, pb.eps, xn, pending)
    qkv_gemm(pb, xn, pb.w_qkv, qkv, pb.b_qkv, qkv_epi, q_scale)
    attend(qkv, o)
    proj_residual_ln2(pb, xs, o, qkv, xn)
    return mlp_residual(pb, x, r0, r1, sc, defer)


def run_block_head(pb: PackedBlock, x: Tensor, r0: int, r1: int, sc: BlockScratch, qkv_epi: Optional[dict],
                   q_scale: float = 0.0) -> None:
    """First half of run_block (LN1 + the QKV GEMM) when the attention is launched separately
    (the global and reloc blocks' attentions paired in one launch)."""
    xs = x[r0:r1]
    xn, qkv = sc.xn[r0:r1], sc.qkv[r0:r1]
    ops.layernorm(xs, pb.ln1_w, pb.ln1_b, pb.eps, xn)
    qkv_gemm(pb, xn, pb.w_qkv, qkv, pb.b_qkv, qkv_epi, q_scale)


def run_block_tail(pb: PackedBlock, x: Tensor, r0: int, r1: int, sc: BlockScratch,
                   defer: bool = False) -> Optional[Pending]:
    """Second half of run_block (proj + residual, LN2, MLP + residual) when the attention
    output sc.o[r0:r1] was produced separately (frame-sharded global block)."""
    xs = x[r0:r1]
    xn, o = sc.xn[r0:r1], sc.o[r0:r1]
    proj_residual_ln2(pb, xs, o, sc.qkv[r0:r1], xn)
    return mlp_residual(pb, x, r0, r1, sc, defer)


# SR_GROUP_TAILS: 0 = never group, 1 = only blocks under GROUP_TAILS_MAX_ROWS rows (a frame-sharded
# rank's 5,496-row global / reloc blocks), 2 = always (default).  Measured, one box each, interleaved:
# G = 2 rank step 213.98 / 213.02 -> 210.87 / 209.69 ms with 2 against 1 (profiles/r05_j12_rs_*.log);
# one GPU level, 79.16 / 79.24 / 79.04 vs 79.20 / 79.09 / 79.20 views/s (r05_j13_bench_g*.log)
_GROUP_TAILS = int(os.environ.get("SR_GROUP_TAILS", "2"))
GROUP_TAILS_MAX_ROWS = 16384


def group_tails_wanted(rows: int) -> bool:
    return _GROUP_TAILS >= 2 or (_GROUP_TAILS == 1 and rows <= GROUP_TAILS_MAX_ROWS)


def run_block_tails(items, x: Tensor, sc: BlockScratch, defer: bool = False) -> list:
    """run_block_tail of several blocks over disjoint row ranges (``items`` = [(pb, r0, r1)]),
    each GEMM stage as ONE sr_gemm_group launch: proj (+LayerScale residual) of every block, the
    LayerNorms, fc1 (+GELU), fc2 (+residual, or deferred).  The per-rank global (anchors) and reloc
    (queries) blocks of a frame-sharded layer are 5,496 rows each at C3 / G = 8: one launch per
    stage fills the CUs that two under-filled ones leave idle.  Per output tile the k order and
    epilogue are those of sr_gemm, so the result does not depend on the grouping.  Returns the
    Pending updates of the deferred fc2 residuals (``defer``)."""
    items = [(pb, r0, r1) for pb, r0, r1 in items if r1 > r0]
    # ``defer`` with every block deferrable: fc2 ends in the bias epilogue into each block's dead
    # attention-output rows sc.o and the updates come back as Pendings (as mlp_residual does alone)
    n_defer = sum(1 for pb, _, _ in items if defer and defer_enabled(pb) and sc.o.shape[1] >= pb.w_fc2.shape[0])
    grouped = (len(items) > 1 and not _FUSED_RESID_LN and n_defer in (0, len(items))
               and all(pb.w_proj is not None and pb.w_fc1 is not None for pb, _, _ in items))
    if grouped:
        hid = [pb.w_fc1.shape[0] for pb, _, _ in items]
        proj = [dict(a=sc.o[r0:r1], w=pb.w_proj, out=x[r0:r1], bias=pb.b_proj, gamma=pb.g1) for pb, r0, r1 in items]
        fc1 = [dict(a=sc.xn[r0:r1], w=pb.w_fc1, out=sc.h[r0:r1, :n], bias=pb.b_fc1)
               for (pb, r0, r1), n in zip(items, hid)]
        if n_defer:
            fc2 = [dict(a=sc.h[r0:r1, :n], w=pb.w_fc2, out=sc.o[r0:r1, :pb.w_fc2.shape[0]], bias=pb.b_fc2)
                   for (pb, r0, r1), n in zip(items, hid)]
        else:
            fc2 = [dict(a=sc.h[r0:r1, :n], w=pb.w_fc2, out=x[r0:r1], bias=pb.b_fc2, gamma=pb.g2)
                   for (pb, r0, r1), n in zip(items, hid)]
        grouped = all(ops.gemm_group_eligible(p) for p in (proj, fc1, fc2))
    if not grouped:
        out = [run_block_tail(pb, x, r0, r1, sc, defer) for pb, r0, r1 in items]
        return [p for p in out if p is not None]
    ops.gemm_group(proj, _lib.SR_EPI_BIAS_RESID, tag="gemm")
    for pb, r0, r1 in items:
        ops.layernorm(x[r0:r1], pb.ln2_w, pb.ln2_b, pb.eps, sc.xn[r0:r1])
    ops.gemm_group(fc1, _lib.SR_EPI_BIAS_GELU, tag="gemm")
    if n_defer:
        ops.gemm_group(fc2, _lib.SR_EPI_BIAS, tag="gemm")
        return [Pending(r0, r1, q["out"], pb.g2) for (pb, r0, r1), q in zip(items, fc2)]
    ops.gemm_group(fc2, _lib.SR_EPI_BIAS_RESID, tag="gemm")
    return []


def frame_attend(pb: PackedBlock, frames: int, tokens: int, tail_readable: bool = False,
                 q_scaled: bool = False) -> Callable[[Tensor, Tensor], None]:
    """Attention within each frame of ``tokens`` rows (attention.py:103 over [B*S, P, C]).
    ``tail_readable``: the qkv buffers come from a Workspace (rows past the last frame readable).
    ``q_scaled``: the QKV GEMM wrote c*q (q_prescale)."""
    C, D = pb.dim, pb.head_dim
    kb, qb = key_norm_bound(pb), query_norm_bound(pb)

    def attend(qkv: Tensor, o: Tensor) -> None:
        ops.attention(qkv[:, 0:C], qkv[:, C:2 * C], qkv[:, 2 * C:3 * C], o, heads=pb.heads, head_dim=D,
                      batch=frames, lq=tokens, q_bstride=tokens, l0=tokens, k0_bstride=tokens, tag="attn_frame",
                      key_norm_max=kb, query_norm_max=qb, tail_readable=tail_readable, q_scaled=q_scaled)
    return attend
