"""Block-level training engine: forward with saved activations ("tape") and backward, on the
HIP kernels (the backward of block.py:86-112 / attention.py:70-122 /
mlp.py:34-40 / layer_scale.py:22-23 that ``loss.backward()`` runs in train_imc.py:404).

Forward (run_block_train) is run_block's kernel sequence with the backward's inputs kept:

    LN1 -> xn1 (+ x0 = x, the same pass)   GEMM qkv -> qkv  (+ aux: pre-norm q|k|v = raw)
    attention(qkv) -> o (+ lse)   GEMM proj + gamma1 + residual (in place on x)
    LN2 -> xn2 (+ x1 = x)   GEMM fc1 + GELU -> h (+ aux: pre-activation u)
    GEMM fc2 + gamma2 + residual

Backward (block_bwd) takes dx (fp32 residual grad of the block output, updated in place to the
grad of its input) and dxb (its bf16 copy, the GEMM operand), and accumulates every parameter
grad into the parameters' ``.grad`` tensors:

    dU  = GELU'(u) * (dxb . (g2 W2))        dgrad GEMM, SR_EPI_GELU_BWD (W^T pack with g2 folded in)
    dW2 = g2 * dxb^T h;  dg2 = <W2, dxb^T h> + b2 * colsum(dx);  db2 = g2 * colsum(dx)
    dxn2 = dU . W1  (fp32);  dW1 = dU^T xn2;  db1 = colsum(dU)
    dx  += LN2'(dxn2; x1)  (+ dxb refresh)   -> the same for proj (o), attention, qk-norm+RoPE, qkv, LN1

Weights for the dgrad GEMMs are packed transposed once per optimizer step (BwdPack).  fp32
blocks (the camera trunk, autocast off) use the same sequence with fp32 GEMMs, the small-row
weight-gradient kernel and the masked fp32 attention backward.
"""

from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Callable, Optional

import torch

from .. import _lib, ops, runtime

Tensor = torch.Tensor


@dataclass
class BlockTape:
    x0: Tensor           # fp32 [R, C]  block input
    x1: Tensor           # fp32 [R, C]  after the attention residual
    xn1: Tensor          # dtype [R, C]
    raw: Tensor          # dtype [R, 3C] pre-norm q|k|v (is qkv when there is no qk-norm / RoPE)
    qkv: Tensor          # dtype [R, 3C]
    o: Tensor            # dtype [R, C]
    lse: Optional[Tensor]  # fp32 [batch*heads*lq] (bf16 attention)
    xn2: Tensor          # dtype [R, C]
    u: Tensor            # dtype [R, H] fc1 pre-activation
    h: Tensor            # dtype [R, H]


TAIL_ROWS = 64
# SR_TRAIN_PAIR_WGRAD (default 1; 0 for the A/B): block_bwd_multi's two items share weight-grad
# launches (ops.gemm_wgrad_pair) where ops.wgrad_pair_splits says it pays
_PAIR_WGRAD = os.environ.get("SR_TRAIN_PAIR_WGRAD", "1") != "0"
# SR_TRAIN_BIAS_COLSUM (bits, default 3; 0 for the A/B): bf16 bias grads from the producing pass
# instead of a column sum that re-reads the gradient: 1 = fc1's from the GELU_BWD dgrad epilogue,
# 2 = qkv's from sr_qk_bwd
_BIAS_COLSUM = int(os.environ.get("SR_TRAIN_BIAS_COLSUM", "3"))
GELU_COLSUM = bool(_BIAS_COLSUM & 1)
QK_COLSUM = bool(_BIAS_COLSUM & 2)


def alloc_tape(rows: int, dim: int, hidden: int, dtype: torch.dtype, device, lse_numel: int,
               separate_raw: bool) -> BlockTape:
    e = lambda r, c, dt=dtype: torch.empty(r, c, device=device, dtype=dt)  # noqa: E731
    # q|k|v with TAIL_ROWS zeroed rows after it: every key segment's tail is readable, so the
    # forward attention may take the hand-scheduled sweep's ragged variant (ops.attention
    # tail_readable; the C4 global block's 21,984 keys are 343.5 tiles)
    qkv = torch.zeros(rows + TAIL_ROWS, 3 * dim, device=device, dtype=dtype)[:rows]
    return BlockTape(x0=e(rows, dim, torch.float32), x1=e(rows, dim, torch.float32), xn1=e(rows, dim),
                     raw=e(rows, 3 * dim) if separate_raw else qkv, qkv=qkv, o=e(rows, dim),
                     lse=torch.empty(lse_numel, device=device, dtype=torch.float32) if lse_numel else None,
                     xn2=e(rows, dim), u=e(rows, hidden), h=e(rows, hidden))


def run_block_train(pb: runtime.PackedBlock, x: Tensor, r0: int, r1: int, tape: BlockTape,
                    attend: Callable[[Tensor, Tensor, Optional[Tensor]], None], qkv_epi: Optional[dict]) -> None:
    """x[r0:r1] <- Block(x[r0:r1]) keeping the backward's inputs in ``tape``."""
    xs = x[r0:r1]
    ops.layernorm(xs, pb.ln1_w, pb.ln1_b, pb.eps, tape.xn1, x_copy=tape.x0)  # x0 = x in the same pass
    if qkv_epi is None:
        ops.gemm(tape.xn1, pb.w_qkv, tape.qkv, _lib.SR_EPI_BIAS, bias=pb.b_qkv, tag="gemm")
    else:
        ops.gemm(tape.xn1, pb.w_qkv, tape.qkv, _lib.SR_EPI_QKV, bias=pb.b_qkv, qkv=qkv_epi, aux=tape.raw, tag="gemm")
    attend(tape.qkv, tape.o, tape.lse)
    ops.gemm(tape.o, pb.w_proj, xs, _lib.SR_EPI_BIAS_RESID, bias=pb.b_proj, gamma=pb.g1, tag="gemm")
    ops.layernorm(xs, pb.ln2_w, pb.ln2_b, pb.eps, tape.xn2, x_copy=tape.x1)  # x1 = x likewise
    ops.gemm(tape.xn2, pb.w_fc1, tape.h, _lib.SR_EPI_BIAS_GELU, bias=pb.b_fc1, aux=tape.u, tag="gemm")
    ops.gemm(tape.h, pb.w_fc2, xs, _lib.SR_EPI_BIAS_RESID, bias=pb.b_fc2, gamma=pb.g2, tag="gemm")


def run_block_train_multi(items) -> None:
    """run_block_train for several independent block applications of equal width at once (the
    layer's reloc and global blocks: different weights, disjoint rows of x, the reloc block's
    anchor K|V already projected): stage by stage in run_block_train's order, each GEMM of all
    items as ONE grouped launch (sr_gemm_group) whose last partial round the items share.  At C4
    each item's N = 1,024 GEMMs (proj, fc2) are 344 tiles of 256^2, which sr_gemm alone runs on
    the 128^2 kernel; grouped they run on the 256^2 kernel, whose results differ from it by fp32
    accumulation order only (gemm_resid 41.7 -> 38.9 ms per C4 step, profiles/r05_j29_*).  fc1
    stays one launch per item.  ``items``: dicts of run_block_train's arguments (pb, x, r0, r1,
    tape, attend, qkv_epi); their attentions run in list order."""
    if len(items) == 1 or not all(it["tape"].xn1.dtype == torch.bfloat16 for it in items) or \
            len({(it["pb"].dim, it["tape"].u.shape[1]) for it in items}) != 1 or \
            len({it["qkv_epi"] is None for it in items}) != 1:
        for it in items:
            run_block_train(it["pb"], it["x"], it["r0"], it["r1"], it["tape"], it["attend"], it["qkv_epi"])
        return

    def group(epi, probs):
        if ops.gemm_group_eligible(probs):
            ops.gemm_group(probs, epi, tag="gemm")
        else:
            for q in probs:
                ops.gemm(q["a"], q["w"], q["out"], epi, bias=q.get("bias"), gamma=q.get("gamma"), qkv=q.get("qkv"),
                         aux=q.get("aux"), tag="gemm")

    for it in items:
        it["_xs"] = it["x"][it["r0"]:it["r1"]]
        ops.layernorm(it["_xs"], it["pb"].ln1_w, it["pb"].ln1_b, it["pb"].eps, it["tape"].xn1, x_copy=it["tape"].x0)
    if items[0]["qkv_epi"] is None:
        group(_lib.SR_EPI_BIAS, [dict(a=it["tape"].xn1, w=it["pb"].w_qkv, out=it["tape"].qkv, bias=it["pb"].b_qkv)
                                 for it in items])
    else:
        group(_lib.SR_EPI_QKV, [dict(a=it["tape"].xn1, w=it["pb"].w_qkv, out=it["tape"].qkv, bias=it["pb"].b_qkv,
                                     qkv=it["qkv_epi"], aux=it["tape"].raw) for it in items])
    for it in items:
        it["attend"](it["tape"].qkv, it["tape"].o, it["tape"].lse)
    group(_lib.SR_EPI_BIAS_RESID, [dict(a=it["tape"].o, w=it["pb"].w_proj, out=it["_xs"], bias=it["pb"].b_proj,
                                        gamma=it["pb"].g1) for it in items])
    for it in items:
        ops.layernorm(it["_xs"], it["pb"].ln2_w, it["pb"].ln2_b, it["pb"].eps, it["tape"].xn2, x_copy=it["tape"].x1)
    for it in items:  # fc1 apart: sr_gemm's tail split beats the group here (35.5 vs 34.9 ms/step, j29)
        ops.gemm(it["tape"].xn2, it["pb"].w_fc1, it["tape"].h, _lib.SR_EPI_BIAS_GELU, bias=it["pb"].b_fc1,
                 aux=it["tape"].u, tag="gemm")
    group(_lib.SR_EPI_BIAS_RESID, [dict(a=it["tape"].h, w=it["pb"].w_fc2, out=it["_xs"], bias=it["pb"].b_fc2,
                                        gamma=it["pb"].g2) for it in items])
    for it in items:
        it.pop("_xs")


# ----------------------------------------------------------------------------- parameters
@dataclass
class BlockGrads:
    """The ``.grad`` tensors of one Block's parameters (fp32, accumulated into)."""
    ln1_w: Tensor
    ln1_b: Tensor
    w_qkv: Tensor
    b_qkv: Optional[Tensor]
    qkn: Optional[Tensor]  # [4, head_dim] = q_norm.weight | q_norm.bias | k_norm.weight | k_norm.bias
    w_proj: Tensor
    b_proj: Optional[Tensor]
    g1: Optional[Tensor]
    ln2_w: Tensor
    ln2_b: Tensor
    w_fc1: Tensor
    b_fc1: Optional[Tensor]
    w_fc2: Tensor
    b_fc2: Optional[Tensor]
    g2: Optional[Tensor]


def _grad(p) -> Optional[Tensor]:
    if p is None:
        return None
    if p.grad is None:
        raise RuntimeError("training engine: parameter grads must be allocated first (train.params.GradBuffer)")
    return p.grad


def block_grads(blk) -> BlockGrads:
    a = blk.attn
    qkn = None
    if getattr(a, "qk_norm", False):
        parts = [a.q_norm.weight.grad, a.q_norm.bias.grad, a.k_norm.weight.grad, a.k_norm.bias.grad]
        if any(t is None for t in parts):
            raise RuntimeError("training engine: qk-norm grads not allocated")
        d = parts[0].numel()
        base = parts[0].data_ptr()
        if any(t.data_ptr() != base + 4 * d * i for i, t in enumerate(parts)):
            raise RuntimeError("training engine: q_norm / k_norm grads must be one contiguous [4, head_dim] block")
        qkn = parts[0].as_strided((4, d), (d, 1))
    ls = lambda m: _grad(getattr(m, "gamma", None))  # noqa: E731
    return BlockGrads(ln1_w=_grad(blk.norm1.weight), ln1_b=_grad(blk.norm1.bias), w_qkv=_grad(a.qkv.weight),
                      b_qkv=_grad(a.qkv.bias), qkn=qkn, w_proj=_grad(a.proj.weight), b_proj=_grad(a.proj.bias),
                      g1=ls(blk.ls1), ln2_w=_grad(blk.norm2.weight), ln2_b=_grad(blk.norm2.bias),
                      w_fc1=_grad(blk.mlp.fc1.weight), b_fc1=_grad(blk.mlp.fc1.bias), w_fc2=_grad(blk.mlp.fc2.weight),
                      b_fc2=_grad(blk.mlp.fc2.bias), g2=ls(blk.ls2))


@dataclass
class BwdPack:
    """Per-optimizer-step transposed weights of one Block for the dgrad GEMMs (dtype), with the
    LayerScale gammas folded into proj / fc2; fp32 masters for the gamma-grad row dots."""
    wt_qkv: Tensor   # [C, 3C]  W_qkv^T
    wt_proj: Tensor  # [C, C]   (g1 * W_proj)^T
    wt_fc1: Tensor   # [C, H]   W_fc1^T
    wt_fc2: Tensor   # [H, C]   (g2 * W_fc2)^T
    w_proj: Tensor   # fp32 masters
    w_fc2: Tensor
    b_proj: Optional[Tensor]
    b_fc2: Optional[Tensor]


def pack_bwd(blk, pb: runtime.PackedBlock, dtype: torch.dtype, into: Optional[BwdPack] = None) -> BwdPack:
    a = blk.attn
    f = lambda t: t.detach()  # noqa: E731  (fp32 contiguous parameters: no copy)
    wq, wp, w1, w2 = f(a.qkv.weight), f(a.proj.weight), f(blk.mlp.fc1.weight), f(blk.mlp.fc2.weight)
    dev = wq.device
    if into is None:
        e = lambda r, c: torch.empty(r, c, device=dev, dtype=dtype)  # noqa: E731
        into = BwdPack(wt_qkv=e(wq.shape[1], wq.shape[0]), wt_proj=e(wp.shape[1], wp.shape[0]),
                       wt_fc1=e(w1.shape[1], w1.shape[0]), wt_fc2=e(w2.shape[1], w2.shape[0]), w_proj=wp, w_fc2=w2,
                       b_proj=pb.b_proj, b_fc2=pb.b_fc2)
    ops.transpose(wq, into.wt_qkv)
    ops.transpose(wp, into.wt_proj, rowscale=pb.g1)
    ops.transpose(w1, into.wt_fc1)
    ops.transpose(w2, into.wt_fc2, rowscale=pb.g2)
    return into


def refresh_items_bf16(blk, pb: runtime.PackedBlock, into: BwdPack) -> list:
    """The block's four weight_refresh items: the bf16 forward weights of the packed block (casts in
    place) and the transposed dgrad packs of pack_bwd (LayerScale gammas folded into proj / fc2)."""
    a = blk.attn
    f = lambda t: t.detach()  # noqa: E731
    return [(f(a.qkv.weight), pb.w_qkv, into.wt_qkv, None),
            (f(a.proj.weight), pb.w_proj, into.wt_proj, pb.g1),
            (f(blk.mlp.fc1.weight), pb.w_fc1, into.wt_fc1, None),
            (f(blk.mlp.fc2.weight), pb.w_fc2, into.wt_fc2, pb.g2)]


def refresh_block_bf16(blk, pb: runtime.PackedBlock, into: BwdPack) -> None:
    """After an optimizer step, one launch per block (sr_weight_refresh_bf16), each fp32 weight read once."""
    ops.weight_refresh(refresh_items_bf16(blk, pb, into))


class BwdScratch:
    """Grow-only backward scratch shared by every block of one stream."""

    def __init__(self):
        self.ws = runtime.Workspace()

    def get(self, name, rows, cols, dtype, device):
        return self.ws.get(name, rows, cols, dtype, device)


def _resid_wants_sum(bias: Optional[Tensor], g_bias: Optional[Tensor], g_gamma: Optional[Tensor]) -> bool:
    return g_bias is not None or (g_gamma is not None and bias is not None)


def _resid_param_grads(dx: Tensor, bias: Optional[Tensor], gamma: Optional[Tensor], g_bias: Optional[Tensor],
                       g_gamma: Optional[Tensor], tmp: Tensor, summed: bool = False) -> None:
    """Bias and LayerScale-gamma grads of ``x += gamma * (a W^T + b)`` from colsum(dx):
    db += gamma * s, dgamma += b * s (the <W, G> part comes from the wgrad row dots).
    ``summed``: tmp already holds colsum(dx) (layernorm_bwd's dx_sum)."""
    if not _resid_wants_sum(bias, g_bias, g_gamma):
        return
    if g_bias is not None and gamma is None:
        raise RuntimeError("bias grad without gamma")
    pairs = ([(g_bias, gamma)] if g_bias is not None else []) + \
        ([(g_gamma, bias)] if g_gamma is not None and bias is not None else [])
    if not summed:  # the column sum's final launch applies the products (no scratch row, no extra launch)
        ops.colsum_fma(dx, pairs)
    elif len(pairs) == 2:
        ops.vec_fma(pairs[0][0], pairs[0][1], tmp, out2=pairs[1][0], a2=pairs[1][1])
    else:
        ops.vec_fma(pairs[0][0], pairs[0][1], tmp)


def block_bwd(pb: runtime.PackedBlock, bp: BwdPack, g: BlockGrads, tape: BlockTape, dx: Tensor,
              dxb: Optional[Tensor], attend_bwd: Callable[[BlockTape, Tensor, Tensor], None],
              qkv_epi: Optional[dict], sc: BwdScratch, tag: str = "bwd") -> None:
    """dx (fp32 [R, C], the grad of the block's output) <- grad of its input, in place; dxb
    (bf16 copy of dx, bf16 blocks) refreshed alongside; parameter grads accumulated.
    ``attend_bwd(tape, dO, dqkv)`` writes fp32 dq|dk|dv into dqkv [R, 3C] (and any shared-segment
    grads elsewhere)."""
    R, C = dx.shape
    Hd = tape.u.shape[1]
    dev = dx.device
    dt = tape.xn1.dtype
    bf = dt == torch.bfloat16
    a_op = dxb if bf else dx   # GEMM operand view of dx
    tmp = sc.get("colsum_tmp", 1, max(C, Hd, 3 * C), torch.float32, dev)[0]

    def wgrad(dy, x, dw, db=None, rowscale=None, wdot=None, rowdot=None):
        if bf:
            ops.gemm_wgrad(dy, x, dw, accumulate=True, rowscale=rowscale, wdot=wdot, rowdot=rowdot, tag=tag + ".wgrad")
            if db is not None:
                ops.colsum(dy, db, accumulate=True)
        else:
            ops.wgrad_small(dy, x, dw, db=db, accumulate=True, rowscale=rowscale, wdot=wdot, rowdot=rowdot)

    # ---- MLP: x2 = x1 + g2 * fc2(GELU(fc1(LN2(x1))))
    dU = sc.get("dU", R, Hd, dt, dev)
    # bf16: fc1's bias grad from the GELU_BWD epilogue's per-64-row column sums (no re-read of dU)
    csU = (sc.get("dU_colsum", ops.colsum_blocks(R), Hd, torch.float32, dev)
           if bf and g.b_fc1 is not None and GELU_COLSUM else None)
    ops.gemm(a_op, bp.wt_fc2, dU, _lib.SR_EPI_GELU_BWD, aux=tape.u, colsum=csU, tag=tag + ".dgrad")
    wgrad(a_op, tape.h, g.w_fc2, rowscale=pb.g2, wdot=bp.w_fc2 if g.g2 is not None else None,
          rowdot=g.g2 if g.g2 is not None else None)
    _resid_param_grads(dx, bp.b_fc2, pb.g2, g.b_fc2, g.g2, tmp[:C])
    dxn = sc.get("dxn", R, C, torch.float32, dev)
    ops.gemm(dU, bp.wt_fc1, dxn, _lib.SR_EPI_F32, tag=tag + ".dgrad")
    wgrad(dU, tape.xn2, g.w_fc1, db=None if csU is not None else g.b_fc1)
    if csU is not None:
        ops.colsum(csU, g.b_fc1, accumulate=True)
    # (LN2's backward also sums the updated dx over the rows: proj's bias / gamma grads below)
    fused_sum = g.ln2_w is not None and C <= 2048 and _resid_wants_sum(bp.b_proj, g.b_proj, g.g1)
    ops.layernorm_bwd(tape.x1, dxn, pb.ln2_w, pb.eps, dx, dxb=dxb, dw=g.ln2_w, db=g.ln2_b,
                      dx_sum=tmp[:C] if fused_sum else None)

    # ---- attention: x1 = x0 + g1 * proj(attn(qk(qkv(LN1(x0)))))
    dO = sc.get("dO", R, C, dt, dev)
    ops.gemm(a_op, bp.wt_proj, dO, _lib.SR_EPI_BIAS, tag=tag + ".dgrad")
    wgrad(a_op, tape.o, g.w_proj, rowscale=pb.g1, wdot=bp.w_proj if g.g1 is not None else None,
          rowdot=g.g1 if g.g1 is not None else None)
    _resid_param_grads(dx, bp.b_proj, pb.g1, g.b_proj, g.g1, tmp[:C], summed=fused_sum)
    dqkv = sc.get("dqkv", R, 3 * C, torch.float32, dev)
    attend_bwd(tape, dO, dqkv)
    if bf:  # (+ the qkv bias grad from the same pass: no bf16 column sum of draw afterwards)
        draw = sc.get("draw", R, 3 * C, dt, dev)
        ops.qk_bwd(tape.raw if qkv_epi is not None else None, dqkv, draw, qkv_epi or dict(embed_dim=C, head_dim=64),
                   grads=g.qkn, bias_grad=g.b_qkv if QK_COLSUM else None)
    elif qkv_epi is not None:  # fp32 block (autocast off) with qk-norm / RoPE: in place on dqkv
        ops.qk_bwd(tape.raw, dqkv, dqkv, qkv_epi, grads=g.qkn)
        draw = dqkv
    else:
        draw = dqkv
    ops.gemm(draw, bp.wt_qkv, dxn, _lib.SR_EPI_F32, tag=tag + ".dgrad")
    wgrad(draw, tape.xn1, g.w_qkv, db=None if bf and QK_COLSUM else g.b_qkv)
    ops.layernorm_bwd(tape.x0, dxn, pb.ln1_w, pb.eps, dx, dxb=dxb, dw=g.ln1_w, db=g.ln1_b)


def block_bwd_multi(items, tag: str = "pair") -> None:
    """block_bwd for several independent block applications of equal width at once (the layer's
    reloc and global blocks: different weights, disjoint rows): stage by stage in block_bwd's
    order, each stage's dgrad GEMMs of all items as ONE grouped launch (sr_gemm_group), whose
    last partial round of workgroups the items share (at C4 each item's N = 1,024 dgrads are
    344 tiles of 256^2, 1.3 rounds alone).  ``items``: dicts of block_bwd's arguments (pb, bp, g,
    tape, dx, dxb, attend_bwd, qkv_epi, sc, tag); their attention backwards run in list order.
    A grouped product runs on the 256^2 kernel with sr_gemm's per-tile order; where sr_gemm
    alone would have picked the 128^2 kernel the results differ by fp32 accumulation order."""
    if len(items) == 1 or not all(it["tape"].xn1.dtype == torch.bfloat16 for it in items) or \
            len({(it["dx"].shape[1], it["tape"].u.shape[1]) for it in items}) != 1:
        for it in items:
            block_bwd(it["pb"], it["bp"], it["g"], it["tape"], it["dx"], it["dxb"], it["attend_bwd"], it["qkv_epi"],
                      it["sc"], tag=it["tag"])
        return
    C = items[0]["dx"].shape[1]
    Hd = items[0]["tape"].u.shape[1]
    dev = items[0]["dx"].device
    dt = torch.bfloat16

    def dgrad(epi, probs):
        if ops.gemm_group_eligible(probs):
            ops.gemm_group(probs, epi, tag=tag + ".dgrad")
        else:
            for q in probs:
                ops.gemm(q["a"], q["w"], q["out"], epi, aux=q.get("aux"), colsum=q.get("colsum"), tag=tag + ".dgrad")

    def wgrad(it, dy, x, dw, db=None, rowscale=None, wdot=None, rowdot=None):
        ops.gemm_wgrad(dy, x, dw, accumulate=True, rowscale=rowscale, wdot=wdot, rowdot=rowdot,
                       tag=it["tag"] + ".wgrad")
        if db is not None:
            ops.colsum(dy, db, accumulate=True)

    def wgrads(args):
        """One stage's weight grads of every item: (it, dy, x, dw, db, rowscale, wdot, rowdot) each;
        two items of one weight shape share one launch where ops.wgrad_pair_splits says it pays."""
        sp = None
        if _PAIR_WGRAD and len(args) == 2 and args[0][3].shape == args[1][3].shape:
            sp = ops.wgrad_pair_splits(args[0][1].shape[0], args[1][1].shape[0], *args[0][3].shape)
        if sp is None:
            for a in args:
                wgrad(*a)
            return
        ops.gemm_wgrad_pair([dict(dy=a[1], x=a[2], dw=a[3], accumulate=True, rowscale=a[5], wdot=a[6], rowdot=a[7])
                             for a in args], sp, tag=tag + ".wgrad")
        for a in args:
            if a[4] is not None:
                ops.colsum(a[1], a[4], accumulate=True)

    for it in items:
        R = it["dx"].shape[0]
        it["_tmp"] = it["sc"].get("colsum_tmp", 1, max(C, Hd, 3 * C), torch.float32, dev)[0]
        it["_dU"] = it["sc"].get("dU", R, Hd, dt, dev)
        it["_csU"] = (it["sc"].get("dU_colsum", ops.colsum_blocks(R), Hd, torch.float32, dev)
                      if it["g"].b_fc1 is not None and GELU_COLSUM else None)
        it["_dxn"] = it["sc"].get("dxn", R, C, torch.float32, dev)
        it["_dO"] = it["sc"].get("dO", R, C, dt, dev)
    # ---- MLP: x2 = x1 + g2 * fc2(GELU(fc1(LN2(x1))))
    dgrad(_lib.SR_EPI_GELU_BWD, [dict(a=it["dxb"], w=it["bp"].wt_fc2, out=it["_dU"], aux=it["tape"].u,
                                      colsum=it["_csU"]) for it in items])
    wgrads([(it, it["dxb"], it["tape"].h, it["g"].w_fc2, None, it["pb"].g2,
             it["bp"].w_fc2 if it["g"].g2 is not None else None, it["g"].g2) for it in items])
    for it in items:
        pb, bp, g = it["pb"], it["bp"], it["g"]
        _resid_param_grads(it["dx"], bp.b_fc2, pb.g2, g.b_fc2, g.g2, it["_tmp"][:C])
    dgrad(_lib.SR_EPI_F32, [dict(a=it["_dU"], w=it["bp"].wt_fc1, out=it["_dxn"]) for it in items])
    wgrads([(it, it["_dU"], it["tape"].xn2, it["g"].w_fc1, None if it["_csU"] is not None else it["g"].b_fc1,
             None, None, None) for it in items])
    for it in items:  # fc1's bias grads from the GELU_BWD epilogue's column sums
        if it["_csU"] is not None:
            ops.colsum(it["_csU"], it["g"].b_fc1, accumulate=True)
    for it in items:
        pb, bp, g = it["pb"], it["bp"], it["g"]
        it["_fused"] = g.ln2_w is not None and C <= 2048 and _resid_wants_sum(bp.b_proj, g.b_proj, g.g1)
        ops.layernorm_bwd(it["tape"].x1, it["_dxn"], pb.ln2_w, pb.eps, it["dx"], dxb=it["dxb"], dw=g.ln2_w,
                          db=g.ln2_b, dx_sum=it["_tmp"][:C] if it["_fused"] else None)
    # ---- attention: x1 = x0 + g1 * proj(attn(qk(qkv(LN1(x0)))))
    dgrad(_lib.SR_EPI_BIAS, [dict(a=it["dxb"], w=it["bp"].wt_proj, out=it["_dO"]) for it in items])
    wgrads([(it, it["dxb"], it["tape"].o, it["g"].w_proj, None, it["pb"].g1,
             it["bp"].w_proj if it["g"].g1 is not None else None, it["g"].g1) for it in items])
    for it in items:
        pb, bp, g = it["pb"], it["bp"], it["g"]
        _resid_param_grads(it["dx"], bp.b_proj, pb.g1, g.b_proj, g.g1, it["_tmp"][:C], summed=it["_fused"])
    for it in items:
        R = it["dx"].shape[0]
        dqkv = it["sc"].get("dqkv", R, 3 * C, torch.float32, dev)
        it["attend_bwd"](it["tape"], it["_dO"], dqkv)
        it["_draw"] = it["sc"].get("draw", R, 3 * C, dt, dev)
        qkv_epi = it["qkv_epi"]
        ops.qk_bwd(it["tape"].raw if qkv_epi is not None else None, dqkv, it["_draw"],
                   qkv_epi or dict(embed_dim=C, head_dim=64), grads=it["g"].qkn,
                   bias_grad=it["g"].b_qkv if QK_COLSUM else None)
    dgrad(_lib.SR_EPI_F32, [dict(a=it["_draw"], w=it["bp"].wt_qkv, out=it["_dxn"]) for it in items])
    wgrads([(it, it["_draw"], it["tape"].xn1, it["g"].w_qkv, None if QK_COLSUM else it["g"].b_qkv, None, None, None)
            for it in items])
    for it in items:
        pb, g = it["pb"], it["g"]
        ops.layernorm_bwd(it["tape"].x0, it["_dxn"], pb.ln1_w, pb.eps, it["dx"], dxb=it["dxb"], dw=g.ln1_w,
                          db=g.ln1_b)


def frame_attend_train(pb: runtime.PackedBlock, frames: int, tokens: int):
    """Forward / backward attention callbacks within each frame (frame and DINO blocks)."""
    C = pb.dim

    def fwd(qkv, o, lse):
        ops.attention(qkv[:, 0:C], qkv[:, C:2 * C], qkv[:, 2 * C:], o, heads=pb.heads, head_dim=pb.head_dim,
                      batch=frames, lq=tokens, q_bstride=tokens, l0=tokens, k0_bstride=tokens, lse=lse,
                      tag="attn_frame", tail_readable=True)

    def bwd(tape, dO, dqkv):
        q = tape.qkv
        delta = _delta(dqkv.device, frames * pb.heads * tokens)
        ops.attention_bwd(q[:, 0:C], q[:, C:2 * C], q[:, 2 * C:], tape.o, tape.lse, dO, dqkv[:, 0:C],
                          dqkv[:, C:2 * C], dqkv[:, 2 * C:], delta, heads=pb.heads, batch=frames, lq=tokens,
                          q_bstride=tokens, l0=tokens, k0_bstride=tokens, tag="attn_bwd_frame")
    return fwd, bwd


_DELTA = {}


def _delta(device, n: int) -> Tensor:
    t = _DELTA.get(device)
    if t is None or t.numel() < n:
        t = torch.empty(n, device=device, dtype=torch.float32)
        _DELTA[device] = t
    return t[:n]
