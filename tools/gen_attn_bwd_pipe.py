#!/usr/bin/env python3
"""Generates self-supervise-sfm_amd/csrc/sr_attn_bwd_pipe.inc: the hand-scheduled query sweep of
attn_bwd_dkdv_pipe_kernel (sr_attn_bwd.hip) as ONE inline-asm statement, for a workgroup of 4
waves with ONE wave per SIMD (launch_bounds(256, 1)); each wave owns 64 keys (two 32-key blocks
kb), so every Q / dO fragment and every lse / delta seed read from LDS feeds both key blocks.

Why: the compiled dK/dV sweep (two waves per SIMD, 256 registers each) reads its MFMA operands
just before use (a ds_read -> s_waitcnt lgkmcnt(0) -> MFMA chain for half the tile) and reaches
about half the MFMA rate.  Per 64-query tile and wave this sweep issues 64 MFMAs (S^T, dP^T, dV^T,
dK^T for two key blocks), 64 v_exp_f32, 64 v_mul_f32 and 64 v_cvt_pk_bf16_f32: about 2,100 cycles
of vector issue beside 2,048 MFMA cycles, so the VALU work must sit in the MFMA gaps.

Software pipeline over the tile's two 32-query blocks A (rows 0-31) and B (rows 32-63), half a
tile apart, so that one block's MFMAs always have the other block's softmax work beside them:

  X(t): MFMA  GR(B, t-1) | SD(B, t)       VALU VAL(A, t)   LDS  tr(A, t), row(A, t+1) | seeds(A, t+1)
  Y(t): MFMA  GR(A, t)   | SD(A, t+1)     VALU VAL(B, t)   LDS  tr(B, t), row(B, t+1), DMA t+3 | seeds(B, t+1)

  SD(q, t):  S^T and dP^T chains of block q (rows: queries, columns: the lane's key) for both key
             blocks, seeded with +lse and -delta: 4 chains x 4 k-steps = 16 MFMAs
  VAL(q, t): P = exp2(-S'), dS = P dP', both packed to bf16 in place: 32 exp, 32 mul, 32 cvt
  GR(q, t):  dV^T += dO^T P, dK^T += Q^T dS over the block's 32 queries: 16 MFMAs

Registers (per lane): S'/dP' of both blocks are named VGPRs (128), packed P / dS overwrite them in
place (into the kb1 halves, order (kb, s2) = (1,0), (1,1), (0,0), (0,1)); one seed set (lse,
-delta: 32 VGPRs) is reloaded at the end of each phase for the next phase's chains (C operand
distinct from D); row fragments (Q, dO rows of a block) and transposed fragments (Q^T, dO^T) are
named AGPRs, one set per block; dK^T / dV^T (128 AGPRs) and the resident K / V fragments (64
VGPRs, K negated and scaled by c) are compiler operands.

The sweep covers the FULL query tiles only (the C++ side runs a ragged last tile afterwards with
the compiled tile body, so the accumulation order -- and every bit of dK / dV -- is the compiled
kernel's).  K/V ring: 4 slots of Q | dO (16 KB) + lse | delta (512 B), tile t+3 staged during tile
t (5 LDS-DMA pieces per wave: 4 rows-pieces + one dword piece of lse / delta).  The loop is
unrolled by the ring depth so every slot is static; LDS addresses are lane-offset operands plus
the instruction's 16-bit offset.

Hazards handled here: lgkmcnt counted per read (LDS returns in order), MFMA -> VALU distance
(valu_lead + s_nop), VALU -> MFMA operand distance, seed reloads only after every chain that
reads them as C has issued its remaining k-steps, M0 -> LDS-DMA s_nop 0, a pad after the last
MFMA.

    python3 tools/gen_attn_bwd_pipe.py     (writes the .inc; committed, regenerate after edits)
"""

import os

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.environ.get("SR_BWD_PIPE_OUT") or os.path.join(HERE, "..", "self-supervise-sfm_amd", "csrc",
                                                        "sr_attn_bwd_pipe.inc")

LV, DV = 96, 112                       # seed set: +lse (16 VGPRs), -delta (16 VGPRs)
NAMED_V = list(range(96, 256))
NAMED_A = list(range(0, 128))
ORDER = [(1, 0), (1, 1), (0, 0), (0, 1)]  # (kb, s2): VALU / packing order
SLOT_B = 16384                         # one ring slot: Q tile | dO tile
TILE_B = 8192
LSE_SLOT = 512                         # lse | delta of one slot (the seed area has its own base)
COST = {"exp": 8, "mul": 4, "cvt": 5, "read": 8, "dma": 16}
# the first VALU of a phase reads S' / dP' that the previous phase's last chains wrote: start it
# after VALU_LEAD MFMAs of this phase and a pad
VALU_LEAD = int(os.environ.get("SR_BWD_PIPE_VALU_LEAD", "2"))
LEAD_NOP = int(os.environ.get("SR_BWD_PIPE_LEAD_NOP", "4"))
X_READS = float(os.environ.get("SR_BWD_PIPE_X_READS", "0.7"))
Y_READS = float(os.environ.get("SR_BWD_PIPE_Y_READS", "0.8"))
# timing-only ablations (WRONG results; for locating the loop's cost): comma list of nobar (no per-tile
# barrier), nodma (no LDS-DMA staging), novalu (no exp / mul / pack), noread (no LDS reads), nowait
# (no lgkmcnt waits)
EXP = set(filter(None, os.environ.get("SR_BWD_PIPE_EXP", "").split(",")))
# the dK/dV sweep's concatenated-items variant (SR_ATTN_BWD_PIPE_ASM_CAT): set while it is generated
CAT = False


def S(q, kb):
    return 128 + 64 * q + 16 * kb


def P(q, kb):
    return 160 + 64 * q + 16 * kb


def FQ(q, s):
    return 32 * q + 4 * s


def FO(q, s):
    return 32 * q + 16 + 4 * s


def TQ(q, s2, db):
    return 64 + 32 * q + 4 * (2 * s2 + db)


def TO(q, s2, db):
    return 64 + 32 * q + 16 + 4 * (2 * s2 + db)


def PP(q, kb, s2):  # packed P of (kb, s2): 4 VGPRs in S(q, 1)
    return S(q, 1) + 4 * ORDER.index((kb, s2))


def PD(q, kb, s2):  # packed dS: 4 VGPRs in P(q, 1)
    return P(q, 1) + 4 * ORDER.index((kb, s2))


def vr(a, n=1):
    return f"v{a}" if n == 1 else f"v[{a}:{a + n - 1}]"


def ar(a, n=1):
    return f"a{a}" if n == 1 else f"a[{a}:{a + n - 1}]"


class Emit:
    """Instruction stream of one tile body with LDS-read bookkeeping: reads are keyed, and an
    MFMA waits (lgkmcnt) for exactly the reads it consumes (LDS returns in issue order)."""

    def __init__(self, pending=()):
        self.lines = []
        self.seq = {}
        self.n = 0
        self.waited = -1
        for k in pending:
            self.seq[k] = self.n
            self.n += 1

    def op(self, s):
        if "nowait" in EXP and s.startswith("s_waitcnt lgkm"):
            return
        if "nobar" in EXP and s == "s_barrier":
            return
        self.lines.append(s)

    def read(self, key, text):
        if "noread" not in EXP:
            self.op(text)
        self.seq[key] = self.n
        self.n += 1

    def wait(self, keys):
        if "noread" in EXP:
            return
        s = max((self.seq[k] for k in keys if k in self.seq), default=-1)
        if s <= self.waited:
            return
        cnt = min(self.n - s - 1, 15)
        self.op(f"s_waitcnt lgkmcnt({cnt})")
        self.waited = self.n - 1 - cnt

    def wait_all(self):
        if "noread" not in EXP and self.waited < self.n - 1:
            self.op("s_waitcnt lgkmcnt(0)")
            self.waited = self.n - 1

    def pending(self):
        return [k for k, s in sorted(self.seq.items(), key=lambda kv: kv[1]) if s > self.waited]


class Phase:
    """One X or Y phase: an ordered MFMA list with VALU and LDS units spread over its gaps by
    issue cost, then the tail units (seed reloads) after the last MFMA."""

    def __init__(self, e):
        self.e = e
        self.mfma = []    # (text, needs)
        self.valu = []    # (cost, [lines])
        self.other = []   # (cost, unit, min_gap)
        self.tail = []    # units

    # ---- MFMA lists
    def sd(self, q):
        """S^T / dP^T chains of block q for both key blocks (kb0 first)."""
        for kb in range(2):
            for which in "SP":
                acc = S(q, kb) if which == "S" else P(q, kb)
                seed = LV if which == "S" else DV
                for s in range(4):
                    a = FQ(q, s) if which == "S" else FO(q, s)
                    b = f"%[k{kb}{s}]" if which == "S" else f"%[v{kb}{s}]"
                    c = vr(seed, 16) if s == 0 else vr(acc, 16)
                    needs = [("row", q, which, s)]
                    if s == 0:
                        needs += [("seed", which, g) for g in range(4)]
                    self.mfma.append((f"v_mfma_f32_32x32x16_bf16 {vr(acc, 16)}, {ar(a, 4)}, {b}, {c}", needs))

    def gr(self, q):
        """dV^T / dK^T of block q: packed (kb, s2) groups in ORDER, both column blocks db."""
        for kb, s2 in ORDER:
            for db in range(2):
                self.mfma.append((f"v_mfma_f32_32x32x16_bf16 %[dv{kb}{db}], {ar(TO(q, s2, db), 4)}, "
                                  f"{vr(PP(q, kb, s2), 4)}, %[dv{kb}{db}]", [("tr", q, "O", s2, db)]))
                self.mfma.append((f"v_mfma_f32_32x32x16_bf16 %[dk{kb}{db}], {ar(TQ(q, s2, db), 4)}, "
                                  f"{vr(PD(q, kb, s2), 4)}, %[dk{kb}{db}]", [("tr", q, "Q", s2, db)]))

    # ---- VALU
    def val(self, q):
        if "novalu" in EXP:
            return
        for kb, s2 in ORDER:
            src, dsp = S(q, kb) + 8 * s2, P(q, kb) + 8 * s2
            for j in range(8):  # P = exp2(-S'), in place
                self.valu.append((COST["exp"], [f"v_exp_f32_e64 {vr(src + j)}, -{vr(src + j)}"]))
            for j in range(8):  # dS = P dP', in place
                self.valu.append((COST["mul"], [f"v_mul_f32_e32 {vr(dsp + j)}, {vr(src + j)}, {vr(dsp + j)}"]))
            pp, pd = PP(q, kb, s2), PD(q, kb, s2)
            for jj in range(4):
                self.valu.append((COST["cvt"], [f"v_cvt_pk_bf16_f32 {vr(pp + jj)}, {vr(src + 2 * jj)}, {vr(src + 2 * jj + 1)}"]))
                self.valu.append((COST["cvt"], [f"v_cvt_pk_bf16_f32 {vr(pd + jj)}, {vr(dsp + 2 * jj)}, {vr(dsp + 2 * jj + 1)}"]))

    # ---- LDS units
    @staticmethod
    def row_units(q, slot):
        out = []
        for s in range(4):
            off = slot * SLOT_B + q * 4096
            out.append([("read", ("row", q, "S", s), f"ds_read_b128 {ar(FQ(q, s), 4)}, %[ra{s}] offset:{off}")])
            out.append([("read", ("row", q, "P", s), f"ds_read_b128 {ar(FO(q, s), 4)}, %[ra{s}] offset:{off + TILE_B}")])
        return out

    @staticmethod
    def tr_units(q, slot):
        out = []
        for s2 in range(2):
            for db in range(2):
                off = slot * SLOT_B + (q * 32 + 16 * s2) * 128
                for which, base, toff in (("O", TO(q, s2, db), TILE_B), ("Q", TQ(q, s2, db), 0)):
                    out.append([("read", ("tr0", q, which, s2, db),
                                 f"ds_read_b64_tr_b16 {ar(base, 2)}, %[ta{db}0] offset:{off + toff}"),
                                ("read", ("tr", q, which, s2, db),
                                 f"ds_read_b64_tr_b16 {ar(base + 2, 2)}, %[ta{db}1] offset:{off + toff}")])
        return out

    @staticmethod
    def seed_units(q, slot):
        out = []
        for which, base, doff in (("S", LV, 0), ("P", DV, 256)):
            for g in range(4):
                off = slot * LSE_SLOT + doff + (q * 32 + 8 * g) * 4
                out.append([("read", ("seed", which, g), f"ds_read_b128 {vr(base + 4 * g, 4)}, %[sa] offset:{off}")])
        return out

    @staticmethod
    def dma_units(slot):
        out = []
        if "nodma" in EXP:
            return out
        for i in range(4):
            out.append([f"s_add_u32 m0, %[ldsv], {slot * SLOT_B + i * 1024}", "s_nop 0",
                        f"global_load_lds_dwordx4 %[dma{i & 1}], %[{'sp' if i < 2 else 'sp2'}]"])
        u = [f"s_add_u32 m0, %[ldsl], {slot * LSE_SLOT}", "s_nop 0", "global_load_lds_dword %[lofs], %[lp]",
             "v_add_u32 %[dma0], %[sstep], %[dma0]", "v_add_u32 %[dma1], %[sstep], %[dma1]"]
        if CAT:
            # items concatenated (one sweep over every item's queries): the lse / -delta of query
            # row r = b lq + i sits at float (b H + h) lq + i, i.e. r + b (H-1) lq past the head's
            # base; b = mulhi(r, M) >> s (exact for r < 2^24, the host's M and s); the next tile's
            # offset is formed right after this tile's copy
            u += ["v_add_u32 %[rrow], 64, %[rrow]", "v_mul_hi_u32 %[tmp], %[rrow], %[mgc]",
                  "v_lshrrev_b32 %[tmp], %[msh], %[tmp]", "v_mul_u32_u24 %[tmp], %[istr], %[tmp]",
                  "v_lshl_add_u32 %[lofs], %[rrow], 2, %[tmp]"]
        else:
            u += ["v_add_u32 %[lofs], 0x100, %[lofs]"]
        out.append(u)
        return out

    def add_other(self, units, cost, min_gap=0):
        for u in units:
            self.other.append((cost * sum(1 for x in u if isinstance(x, tuple) or x.startswith(("ds_", "global_"))),
                               u, min_gap))

    # ---- emission
    def _run(self, unit):
        for x in unit:
            if isinstance(x, tuple):
                _, key, text = x
                self.e.read(key, text)
            else:
                self.e.op(x)

    def emit(self, valu_lead=VALU_LEAD, lead_nop=LEAD_NOP, other_frac=0.7, all_other_first=False):
        nm = len(self.mfma)
        sched = {g: [] for g in range(-1, nm)}
        if self.other:
            if all_other_first:
                for _, u, _ in self.other:
                    sched[-1].append(u)
            else:
                og = max(1, int(round(nm * other_frac)))
                tot = sum(c for c, _, _ in self.other)
                acc = 0.0
                for c, u, mg in self.other:
                    g = max(mg - 1, min(og - 1, int(acc / tot * og)) - 1)
                    sched[g].append(u)
                    acc += c
        if self.valu:
            first_gap = min(valu_lead, nm) - 1
            vg = nm - first_gap
            tot = sum(c for c, _ in self.valu)
            acc = 0.0
            for i, (c, lines) in enumerate(self.valu):
                g = first_gap + min(vg - 1, int(acc / tot * vg))
                if i == 0 and lead_nop:
                    sched[g].append([f"s_nop {lead_nop}"])
                sched[g].append(lines)
                acc += c
        for u in sched[-1]:
            self._run(u)
        for g, (text, needs) in enumerate(self.mfma):
            self.e.wait(needs)
            self.e.op(text)
            for u in sched[g]:
                self._run(u)
        for u in self.tail:
            self._run(u)


def body(t4, pending, first=False, stage=True, vm=5, last=False):
    """Tile t with t % 4 == t4 (ring slot t4).  Returns (lines, pending reads at the end)."""
    e = Emit(pending)
    cur, nxt, stg = t4, (t4 + 1) & 3, (t4 + 3) & 3
    e.op(f"; ---- tile body slot {t4} first={int(first)} stage={int(stage)} vmcnt={vm} last={int(last)}")
    # tile t+1 landed (tile t+2's five pieces may stay in flight); every wave is done with slot t-1
    e.op(f"s_waitcnt vmcnt({vm})")
    e.op("s_barrier")
    if first:
        # fill: block A's chains of tile 0; block B's rows and seeds for X(0)
        p = Phase(e)
        for u in Phase.row_units(0, cur) + Phase.row_units(1, cur) + Phase.seed_units(0, cur):
            p.other.append((0, u, 0))
        p.sd(0)
        p.tail = Phase.seed_units(1, cur)
        p.emit(all_other_first=True)
    # X(t)
    p = Phase(e)
    if not first:
        p.gr(1)
    p.sd(1)
    p.val(0)
    p.add_other(Phase.tr_units(0, cur), COST["read"], 0)
    if not last:
        p.add_other(Phase.row_units(0, nxt), COST["read"], 3)
        p.tail = Phase.seed_units(0, nxt)
    p.emit(other_frac=X_READS)
    # Y(t)
    p = Phase(e)
    p.gr(0)
    if not last:
        p.sd(0)
    p.val(1)
    p.add_other(Phase.tr_units(1, cur), COST["read"], 0)
    if not last:
        p.add_other(Phase.row_units(1, nxt), COST["read"], 3)
    if stage:
        for u in Phase.dma_units(stg):
            p.other.append((COST["dma"], u, 2))
    if not last:
        p.tail = Phase.seed_units(1, nxt)
    p.emit(other_frac=Y_READS)
    if last:
        # GR(B, t): its packed operands were just written by VAL(B, t) (VALU -> MFMA operand)
        e.op("s_nop 4")
        p = Phase(e)
        p.gr(1)
        p.emit()
        e.wait_all()
        return e.lines, []
    # the seed reloads (the tail) stay in flight across the body boundary; every other read is
    # complete here (issued early in Y, so the wait costs nothing)
    last_other = max((s for k, s in e.seq.items() if k[0] != "seed" and s > e.waited), default=-1)
    if last_other > e.waited:
        e.wait([k for k, s in e.seq.items() if s == last_other])
    return e.lines, e.pending()


def sweep():
    L = lambda n: f"{n}_%="  # noqa: E731  (%= : a number unique to the asm statement instance)
    lines = ["s_nop 4", "s_waitcnt lgkmcnt(0)"]  # fresh readfirstlane scalars -> global_load bases
    b, pend = body(0, [], first=True)
    lines += b
    steady = pend
    lines += [f"{L('Lgrp')}:", "s_cmp_eq_u32 %[n], 0", f"s_cbranch_scc1 {L('Lrem')}"]
    loop = []
    for t4 in (1, 2, 3, 0):
        b, p2 = body(t4, pend)
        assert p2 == steady, (t4, p2, steady)
        loop += b
    lines += loop
    lines += ["s_sub_u32 %[n], %[n], 1", f"s_branch {L('Lgrp')}", f"{L('Lrem')}:"]
    for r in range(4):
        lines += [f"s_cmp_eq_u32 %[rem], {r}", f"s_cbranch_scc1 {L(f'Lr{r}')}"]
    for r in range(4):
        lines += [f"{L(f'Lr{r}')}:"]
        for k in range(r):
            b, p2 = body(1 + k, pend)
            assert p2 == steady
            lines += b
        t0 = 1 + r
        b, p2 = body(t0 & 3, pend, stage=False, vm=5)
        assert p2 == steady
        lines += b
        b, p2 = body((t0 + 1) & 3, pend, stage=False, vm=0)
        assert p2 == steady
        lines += b
        b, _ = body((t0 + 2) & 3, pend, stage=False, vm=0, last=True)
        lines += b
        lines += [f"s_branch {L('Ldone')}"]
    lines += [f"{L('Ldone')}:"]
    # the compiler reads dK / dV right after the statement (XDL write -> read): pad
    lines += ["s_nop 15", "s_nop 15"]
    return lines, loop


# ======================================================================== dQ sweep
# attn_bwd_dq_pipe_kernel: each wave owns 64 queries (blocks A, B of 32; lane = the block's query
# l32), the workgroup 256; key tiles of 64 stream through the ring (K tile | V tile).  Per tile
# and block:  SD: S'^T = K (cQ)^T - lse and dP'^T = V dO^T - delta, two key blocks kb each (16
# MFMAs; the K / V row fragments are read once for both query blocks);  VAL: dS = exp2(S') dP',
# packed to bf16 in place (32 exp, 32 mul, 16 cvt);  GR: dQ^T += K^T dS^T (8 MFMAs, in the
# compiled kernel's (kb, s2) order).  The same half-tile pipeline as the dK/dV sweep:
#   X(t): MFMA GR(B, t-1) | SD(B, t)   VALU VAL(A, t)   LDS K rows(t+1) after SD(B, t)'s S chains | V rows(t+1)
#   Y(t): MFMA GR(A, t)   | SD(A, t+1) VALU VAL(B, t)   LDS K^T(t+1) (the other parity set)
# The row fragments are single-buffered (64 AGPRs), K^T double-buffered by tile parity (64 AGPRs);
# dQ^T (64 AGPRs), c q and dO (64 AGPRs) and the -lse / -delta seeds (64 VGPRs) are operands.


def FK(kb, s):
    return 4 * (4 * kb + s)


def FV(kb, s):
    return 32 + 4 * (4 * kb + s)


def KT(par, kb, s2, db):
    return 64 + 32 * par + 4 * (4 * kb + 2 * s2 + db)


class DqPhase(Phase):
    def sd(self, q):
        for which in "SP":
            for kb in range(2):
                acc = S(q, kb) if which == "S" else P(q, kb)
                for s in range(4):
                    a = FK(kb, s) if which == "S" else FV(kb, s)
                    b = f"%[q{q}{s}]" if which == "S" else f"%[o{q}{s}]"
                    c = (f"%[nl{q}]" if which == "S" else f"%[nd{q}]") if s == 0 else vr(acc, 16)
                    key = ("krow", kb, s) if which == "S" else ("vrow", kb, s)
                    self.mfma.append((f"v_mfma_f32_32x32x16_bf16 {vr(acc, 16)}, {ar(a, 4)}, {b}, {c}", [key]))

    def gr(self, q, par):
        for kb in range(2):
            for s2 in range(2):
                for db in range(2):
                    self.mfma.append((f"v_mfma_f32_32x32x16_bf16 %[dq{q}{db}], {ar(KT(par, kb, s2, db), 4)}, "
                                      f"{vr(PD(q, kb, s2), 4)}, %[dq{q}{db}]", [("kt", par, kb, s2, db)]))

    def val(self, q):
        if "novalu" in EXP:
            return
        for kb, s2 in ORDER:
            src, dsp = S(q, kb) + 8 * s2, P(q, kb) + 8 * s2
            for j in range(8):  # P = exp2(S'), in place
                self.valu.append((COST["exp"], [f"v_exp_f32_e32 {vr(src + j)}, {vr(src + j)}"]))
            for j in range(8):  # dS = P dP', in place
                self.valu.append((COST["mul"], [f"v_mul_f32_e32 {vr(dsp + j)}, {vr(src + j)}, {vr(dsp + j)}"]))
            pd = PD(q, kb, s2)
            for jj in range(4):
                self.valu.append((COST["cvt"], [f"v_cvt_pk_bf16_f32 {vr(pd + jj)}, {vr(dsp + 2 * jj)}, {vr(dsp + 2 * jj + 1)}"]))

    @staticmethod
    def row_units(which, slot):
        out = []
        for kb in range(2):
            for s in range(4):
                if which == "K":
                    out.append([("read", ("krow", kb, s),
                                 f"ds_read_b128 {ar(FK(kb, s), 4)}, %[ra{s}] offset:{slot * SLOT_B + kb * 4096}")])
                else:
                    out.append([("read", ("vrow", kb, s),
                                 f"ds_read_b128 {ar(FV(kb, s), 4)}, %[ra{s}] offset:{slot * SLOT_B + TILE_B + kb * 4096}")])
        return out

    @staticmethod
    def kt_units(slot, par):
        out = []
        for kb in range(2):
            for s2 in range(2):
                for db in range(2):
                    off = slot * SLOT_B + (kb * 32 + 16 * s2) * 128
                    base = KT(par, kb, s2, db)
                    out.append([("read", ("kt0", par, kb, s2, db), f"ds_read_b64_tr_b16 {ar(base, 2)}, %[ta{db}0] offset:{off}"),
                                ("read", ("kt", par, kb, s2, db), f"ds_read_b64_tr_b16 {ar(base + 2, 2)}, %[ta{db}1] offset:{off}")])
        return out

    @staticmethod
    def dq_dma_units(slot, pieces):
        out = []
        if "nodma" in EXP:
            return out
        for i in pieces:
            u = [f"s_add_u32 m0, %[ldsv], {slot * SLOT_B + i * 1024}", "s_nop 0",
                 f"global_load_lds_dwordx4 %[dma{i & 1}], %[{'sp' if i < 2 else 'sp2'}]"]
            if i == 3:
                u += ["v_add_u32 %[dma0], %[sstep], %[dma0]", "v_add_u32 %[dma1], %[sstep], %[dma1]"]
            out.append(u)
        return out


def dq_body(t4, first=False, stage=True, vm=4, last=False):
    e = Emit()
    cur, nxt, stg = t4, (t4 + 1) & 3, (t4 + 3) & 3
    par = t4 & 1
    e.op(f"; ---- dQ tile body slot {t4} first={int(first)} stage={int(stage)} vmcnt={vm} last={int(last)}")
    e.op(f"s_waitcnt vmcnt({vm})")  # tile t+1 landed (tile t+2's four pieces may stay in flight)
    e.op("s_barrier")
    if first:
        p = DqPhase(e)
        for u in DqPhase.row_units("K", cur) + DqPhase.row_units("V", cur) + DqPhase.kt_units(cur, par):
            p.other.append((0, u, 0))
        p.sd(0)
        p.emit(all_other_first=True)
    # X(t)
    p = DqPhase(e)
    if not first:
        p.gr(1, par ^ 1)
    n_gr = len(p.mfma)
    p.sd(1)
    p.val(0)
    if not last:
        p.add_other(DqPhase.row_units("K", nxt), COST["read"], n_gr + 8)  # after SD(B, t)'s S chains
        p.tail = DqPhase.row_units("V", nxt)
    if stage:
        for u in DqPhase.dq_dma_units(stg, (0, 1)):
            p.other.append((COST["dma"], u, 2))
    p.emit(other_frac=1.0)
    # Y(t)
    p = DqPhase(e)
    p.gr(0, par)
    if not last:
        p.sd(0)
        p.add_other(DqPhase.kt_units(nxt, par ^ 1), COST["read"], 0)
    p.val(1)
    if stage:
        for u in DqPhase.dq_dma_units(stg, (2, 3)):
            p.other.append((COST["dma"], u, 2))
    p.emit(other_frac=Y_READS)
    if last:
        e.op("s_nop 4")
        p = DqPhase(e)
        p.gr(1, par)
        p.emit()
    e.wait_all()
    return e.lines


def dq_sweep():
    L = lambda n: f"{n}_%="  # noqa: E731
    lines = ["s_nop 4", "s_waitcnt lgkmcnt(0)"]
    lines += dq_body(0, first=True)
    lines += [f"{L('Lgrp')}:", "s_cmp_eq_u32 %[n], 0", f"s_cbranch_scc1 {L('Lrem')}"]
    loop = []
    for t4 in (1, 2, 3, 0):
        loop += dq_body(t4)
    lines += loop
    lines += ["s_sub_u32 %[n], %[n], 1", f"s_branch {L('Lgrp')}", f"{L('Lrem')}:"]
    for r in range(4):
        lines += [f"s_cmp_eq_u32 %[rem], {r}", f"s_cbranch_scc1 {L(f'Lr{r}')}"]
    for r in range(4):
        lines += [f"{L(f'Lr{r}')}:"]
        for k in range(r):
            lines += dq_body(1 + k)
        t0 = 1 + r
        lines += dq_body(t0 & 3, stage=False, vm=4) + dq_body((t0 + 1) & 3, stage=False, vm=0)
        lines += dq_body((t0 + 2) & 3, stage=False, vm=0, last=True)
        lines += [f"s_branch {L('Ldone')}"]
    lines += [f"{L('Ldone')}:", "s_nop 15", "s_nop 15"]
    return lines, loop


def stats(name, lines, loop):
    n_mfma = sum(1 for l in loop if l.startswith("v_mfma")) // 4
    n_valu = sum(1 for l in loop if l.startswith(("v_exp", "v_mul", "v_cvt"))) // 4
    n_ds = sum(1 for l in loop if l.startswith("ds_")) // 4
    n_wait = sum(1 for l in loop if l.startswith("s_waitcnt lgkm")) // 4
    n_all = sum(1 for l in loop if not l.startswith(";") and not l.endswith(":")) // 4
    return (f"{name}: per tile {n_mfma} MFMA, {n_valu} exp/mul/pack VALU, {n_ds} LDS reads, {n_wait} lgkmcnt "
            f"waits, {n_all} instructions; {len(lines)} asm lines")


def cat_sweep():
    global CAT
    CAT = True
    try:
        return sweep()
    finally:
        CAT = False


def main():
    out = ["// GENERATED by tools/gen_attn_bwd_pipe.py — do not edit by hand."]
    for name, (lines, loop) in (("SR_ATTN_BWD_PIPE_ASM", sweep()), ("SR_ATTN_BWD_PIPE_ASM_CAT", cat_sweep()),
                                ("SR_ATTN_BWD_DQ_ASM", dq_sweep())):
        st = stats(name, lines, loop)
        print(st)
        out.append("// " + st)
        out.append(f"#define {name} \\")
        out.append(" \\\n".join("  \"" + l + "\\n\\t\"" for l in lines))
    clob = ", ".join([f'"v{r}"' for r in NAMED_V] + [f'"a{r}"' for r in NAMED_A])
    out.append("#define SR_ATTN_BWD_PIPE_CLOBBERS " + clob)
    clob = ", ".join([f'"v{r}"' for r in range(128, 256)] + [f'"a{r}"' for r in range(0, 128)])
    out.append("#define SR_ATTN_BWD_DQ_CLOBBERS " + clob)
    with open(OUT, "w") as f:
        f.write("\n".join(out) + "\n")


if __name__ == "__main__":
    main()
