#!/usr/bin/env python3
"""Generates self-supervise-sfm_amd/csrc/sr_attn_pipe.inc: the hand-scheduled K/V sweep of
attn_bf16_kernel<4, 2, KIND, PIPE=true> (sr_attn.hip) as ONE inline-asm statement, for a
workgroup of 4 waves with ONE wave per SIMD (launch_bounds(256, 1): the whole 512-entry register
file per lane, so the sweep keeps every fragment it reads).

Why: at head_dim 64 the loop is issue-bound (MI355X_MICROARCH.md constants: v_exp_f32 8 cycles of
a SIMD's vector issue, v_cvt_pk 4-5, an MFMA 8 of its 32; per wave and 64-key tile 64 exp2 + 32
packs beside 32 + 8 MFMAs), and two waves per SIMD share one issue port.  One wave per SIMD
issues its own exp2 / pack stretch into its own MFMA gaps, with the wave's two q-blocks half a
tile apart so that one q-block's MFMAs always have the other's VALU beside them:

  X(t): MFMA  QK1(t) kb0 | PV1(t-1) | QK1(t) kb1     VALU EXP0(t)   LDS K(t+1) -> Kset[t+1], V(t) -> Vset[t]
  Y(t): MFMA  QK0(t+1) kb0 | PV0(t) | QK0(t+1) kb1   VALU EXP1(t)   LDS-DMA of tile t+3

Fixed offset m per query row (exp2 domain): every q.k^T chain starts from the accumulator
operand %[mn<b>] = -m broadcast (16 VGPRs per q-block), so P = exp2(S) needs no max tracking;
the C++ side picks m from the row's Cauchy-Schwarz bound (m = 0 when it is <= 64) and checks it
against tile 0's row max.

Every K and V fragment of a tile is read from LDS ONCE (into AGPR sets, double-buffered by tile
parity) and used by both q-blocks.  Scores S_b (32 VGPRs per q-block) are named VGPRs; P
overwrites its own scores in place (S_b[16:31], EXP order (1,0),(1,1),(0,0),(0,1)).  O, Q and
the row sums are compiler-allocated AGPR operands.  K/V ring: 4 stages of 16 KB, tile t+3 staged
during tile t (its slot last read in X(t-1)).  The loop is unrolled by the ring depth, so every
tile's slot (and register parity) is static: LDS fragment addresses are six lane-offset operands
plus the instruction's 16-bit offset, with no per-tile address arithmetic; four tail variants (by
(ntiles - 4) % 4) end the sweep.

Hazards handled here: lgkmcnt counted per fragment read (LDS returns in order), MFMA -> VALU
(scores) and VALU -> MFMA (P) distances, M0 -> LDS-DMA s_nop 0, and the trailing pad before the
compiler reads O / l.

    python3 tools/gen_attn_pipe.py          (writes the .inc; committed, regenerate after edits)

Three statements: SR_ATTN_PIPE_ASM (one segment of whole tiles), SR_ATTN_PIPE_ASM_SEG (two segments,
ragged tails) and SR_ATTN_PIPE_ASM_VT (as the first, V staged pre-transposed: see VT below).
"""

import os

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.environ.get("SR_PIPE_OUT") or os.path.join(HERE, "..", "self-supervise-sfm_amd", "csrc", "sr_attn_pipe.inc")

S = {0: 160, 1: 192}          # S_b: 32 VGPRs, kb block k at S_b + 16k
NAMED_V = list(range(160, 224))
# LDS addresses are lane offsets in operands (%[ka0..3] = lds0 + koff[s], %[va0..1] = lds0 +
# voff[db]); the ring slot of a tile is static per body (the loop is unrolled by the ring depth),
# so slot, K-block and V row offsets all ride in the instructions' 16-bit offset field
KSET = [0, 32]                # AGPR bases: K fragment (kb, s) at KSET[p] + 4 (4 kb + s)
VSET = [64, 96]               # AGPR bases: V^T fragment (i, db) at VSET[p] + 4 (2 i + db)
NAMED_A = list(range(0, 128))
EXP_ORDER = [(1, 0), (1, 1), (0, 0), (0, 1)]  # (kb, s2) in EXP / P-fragment order
TILE_B = 8192
STAGE_B = 2 * TILE_B
# issue cost weights (cycles of the SIMD's vector issue; MI355X_MICROARCH.md constants table)
COST = {"exp": int(os.environ.get("SR_PIPE_EXP_COST", "8")), "cvt": 5, "read": 8, "dma": 16}
# tuning knobs (A/B builds; the defaults are the measured best):
#   SR_PIPE_DMA_IN_X=1: LDS-DMA of tile t+3 in X and V(t) reads at the head of Y (measured slower:
#   global 6.52-6.57 vs 6.39-6.41 ms with V(t) in X and the DMA in Y)
#   SR_PIPE_X_READS / SR_PIPE_Y_DMA: share of a phase's MFMA gaps the reads / DMA pieces spread over
DMA_IN_X = os.environ.get("SR_PIPE_DMA_IN_X", "0") != "0"
X_READS = float(os.environ.get("SR_PIPE_X_READS", "0.6"))
Y_DMA = float(os.environ.get("SR_PIPE_Y_DMA", "0.8"))
# XDL write -> VALU read of the same VGPR needs 11 wait states (8-pass 32x32x16): X's first exp2
# reads the scores Y's last MFMA chain wrote ~10 instructions earlier, so pad
X_LEAD_NOP = int(os.environ.get("SR_PIPE_X_LEAD_NOP", "2"))
#   SR_PIPE_K1_IN_Y=1: K(t+1)'s kb1 fragments read at the head of Y (its chain is Y's last) instead of in X
#   SR_PIPE_DMA_SPLIT=k: the first k DMA pieces in X, the rest in Y
K1_IN_Y = os.environ.get("SR_PIPE_K1_IN_Y", "0") == "1"
DMA_SPLIT = int(os.environ.get("SR_PIPE_DMA_SPLIT", "0"))
# SR_ATTN_PIPE_ASM_SEG (generated with SEG = True): two key segments (the DMA source switches to
# segment 1's base, offsets and tile stride when tile nt0 is staged: %[nsw] = nt0 - 3) and ragged
# segment tails (scores of keys past a segment's end -> -inf before their exp2: tiles %[trag0] /
# %[trag1], per-lane valid-key thresholds %[vk0] / %[vk1] = valid - 4 hi).  The staging then reads
# up to 63 rows past a segment's end: the caller guarantees them readable and finite.
SEG = False
# SR_ATTN_PIPE_ASM_VT (generated with VT = True): the V half of each stage holds the V^T tile
# (sr_vt_tiles: 64 rows d x 64 key slots in the P fragment's k order, staged with K's swizzle), so a
# V^T fragment is ONE ds_read_b128 at a K-fragment lane address (%[ka<2 kb + s2>], +4096 for d block
# 1) instead of two ds_read_b64_tr_b16
VT = False
_LABEL = [0]


def _label(stem):
    _LABEL[0] += 1
    return f"L{stem}{_LABEL[0]}_%="


# timing-only experiments (WRONG results: they race the K/V ring): no per-tile barrier / a vmcnt
# wait one tile looser
NO_BARRIER = os.environ.get("SR_PIPE_EXP_NO_BARRIER") == "1"
VM_SLACK = int(os.environ.get("SR_PIPE_EXP_VM_SLACK", "0"))
# timing-only (WRONG results): V fragments as one conflict-free ds_read_b128 each (what a V^T tile
# would cost) / two LDS-DMA pieces per wave and tile instead of four
EXP_VB128 = os.environ.get("SR_PIPE_EXP_VB128") == "1"
EXP_DMA2 = os.environ.get("SR_PIPE_EXP_DMA2") == "1"


def vr(a, n=1):
    return f"v{a}" if n == 1 else f"v[{a}:{a + n - 1}]"


def ar(a, n=1):
    return f"a{a}" if n == 1 else f"a[{a}:{a + n - 1}]"


def kfrag(p, kb, s):
    return KSET[p] + 4 * (4 * kb + s)


def vfrag(p, i, db):
    return VSET[p] + 4 * (2 * i + db)


class Emit:
    def __init__(self):
        self.lines = []
        self.reads = 0       # LDS reads issued (sequence numbers)
        self.waited = -1     # highest read sequence known complete

    def op(self, s):
        self.lines.append(s)

    def ds(self, s):
        self.op(s)
        self.reads += 1
        return self.reads - 1

    def wait_read(self, seq):
        if seq is None or seq <= self.waited:
            return
        n = self.reads - seq - 1
        self.op(f"s_waitcnt lgkmcnt({min(n, 15)})")
        self.waited = seq

    def wait_all_reads(self):
        if self.waited < self.reads - 1:
            self.op("s_waitcnt lgkmcnt(0)")
            self.waited = self.reads - 1


class Phase:
    """One X or Y phase: an ordered MFMA list interleaved with filler units (VALU, LDS reads,
    LDS-DMA pieces), spread over the MFMA gaps by issue cost."""

    def __init__(self, e):
        self.e = e
        self.mfma = []     # (kind, params)
        self.valu = []     # (cost, [lines])
        self.other = []    # (cost, [lines], kind) reads / dma, issued early

    # ---- MFMA lists
    def qk(self, b, kb, p):
        for s in range(4):
            self.mfma.append(("qk", (b, kb, s, p)))

    def pv(self, b, p):
        for i, (kb, s2) in enumerate(EXP_ORDER):
            self.mfma.append(("rs", (b, i)))
            for db in range(2):
                self.mfma.append(("pv", (b, i, db, p)))

    # ---- fillers
    def exp(self, b):
        base = S[b]
        for i, (kb, s2) in enumerate(EXP_ORDER):
            src = base + 16 * kb + 8 * s2
            for j in range(8):
                self.valu.append((COST["exp"], [f"v_exp_f32 {vr(src + j)}, {vr(src + j)}"]))
            dst = base + 16 + 4 * i
            for jj in range(4):
                self.valu.append((COST["cvt"], [f"v_cvt_pk_bf16_f32 {vr(dst + jj)}, {vr(src + 2 * jj)}, "
                                                f"{vr(src + 2 * jj + 1)}"]))

    def read_k(self, p, slot, seqs, kbs=(0, 1)):
        """K fragments of the tile in ring slot `slot` into Kset[p] (8 ds_read_b128)."""
        for kb in kbs:
            for s in range(4):
                lines = [("ds", f"ds_read_b128 {ar(kfrag(p, kb, s), 4)}, %[ka{s}] "
                                f"offset:{slot * STAGE_B + kb * 4096}", seqs, (p, kb, s))]
                self.other.append((COST["read"], lines, "read"))

    def read_v(self, p, slot, seqs):
        """V^T fragments of the tile in ring slot `slot` into Vset[p] (16 ds_read_b64_tr_b16)."""
        for i, (kb, s2) in enumerate(EXP_ORDER):
            for db in range(2):
                off = slot * STAGE_B + TILE_B + (kb * 32 + 16 * s2) * 128
                f = vfrag(p, i, db)
                if VT:
                    lines = [("ds", f"ds_read_b128 {ar(f, 4)}, %[ka{2 * kb + s2}] "
                                    f"offset:{slot * STAGE_B + TILE_B + db * 4096}", seqs, (p, i, db))]
                    self.other.append((COST["read"], lines, "read"))
                    continue
                if EXP_VB128:
                    lines = [("ds", f"ds_read_b128 {ar(f, 4)}, %[ka{(2 * i + db) & 3}] "
                                    f"offset:{slot * STAGE_B + TILE_B + (i >> 1) * 4096}", seqs, (p, i, db))]
                    self.other.append((COST["read"], lines, "read"))
                    continue
                lines = [("ds", f"ds_read_b64_tr_b16 {ar(f, 2)}, %[va{db}] offset:{off}", None, None),
                         ("ds", f"ds_read_b64_tr_b16 {ar(f + 2, 2)}, %[va{db}] offset:{off + 1024}", seqs, (p, i, db))]
                self.other.append((2 * COST["read"], lines, "read"))

    def dma(self, slot, pieces=range(4)):
        """LDS-DMA of tile t+3 (4 pieces of 8 rows per wave) into ring slot `slot`; the per-lane
        source offsets then step one tile."""
        step = "%[sstc]" if SEG else "%[sstep]"
        if EXP_DMA2:
            pieces = [i for i in pieces if i in (0, 3)]
        for i in pieces:
            lines = []
            if SEG and i == 0:
                sk = _label("sw")
                lines += ["s_cmp_eq_u32 %[tcur], %[nsw]", f"s_cbranch_scc0 {sk}",
                          "s_mov_b64 %[sp], %[sp1]", "s_mov_b64 %[sp2], %[sp1b]", "s_mov_b32 %[sstc], %[sstep1]",
                          "v_mov_b32 %[dma0], %[dm10]", "v_mov_b32 %[dma1], %[dm11]", f"{sk}:"]
            lines += [f"s_add_u32 m0, %[ldsv], {slot * STAGE_B + i * 1024}", "s_nop 0",
                      f"global_load_lds_dwordx4 %[dma{i & 1}], %[{'sp' if i < 2 else 'sp2'}]"]
            if i == 3:
                lines += [f"v_add_u32 %[dma0], {step}, %[dma0]", f"v_add_u32 %[dma1], {step}, %[dma1]"]
            self.other.append((COST["dma"], lines, "dma"))

    # ---- emission
    def _issue_mfma(self, m, kseqs, vseqs):
        kind, p = m
        e = self.e
        if kind == "qk":
            b, kb, s, ps = p
            e.wait_read(kseqs.get((ps, kb, s)))
            acc = vr(S[b] + 16 * kb, 16)
            # the chain starts from -m (the row's fixed offset, broadcast over the lane's 16
            # accumulator entries: every entry of a lane is a score of ONE query row), so the
            # chain returns c q.k - m with no fold MFMA and no per-score subtraction
            c = f"%[mn{b}]" if s == 0 else acc
            e.op(f"v_mfma_f32_32x32x16_bf16 {acc}, {ar(kfrag(ps, kb, s), 4)}, %[q{b}{s}], {c}")
        elif kind == "rs":
            b, i = p
            e.op(f"v_mfma_f32_16x16x32_bf16 %[l{b}], %[suma], {vr(S[b] + 16 + 4 * i, 4)}, %[l{b}]")
        else:
            b, i, db, ps = p
            e.wait_read(vseqs.get((ps, i, db)))
            e.op(f"v_mfma_f32_32x32x16_bf16 %[o{b}{db}], {ar(vfrag(ps, i, db), 4)}, {vr(S[b] + 16 + 4 * i, 4)}, "
                 f"%[o{b}{db}]")

    def _emit_unit(self, lines):
        for ln in lines:
            if isinstance(ln, tuple):
                _, text, seqs, key = ln
                seq = self.e.ds(text)
                if seqs is not None:
                    seqs[key] = seq
            else:
                self.e.op(ln)

    def emit(self, kseqs, vseqs, valu_lead=0, lead_nop=0, other_frac=0.6):
        """Reads / DMA pieces are spread over the first other_frac of the gaps, VALU over the gaps
        after MFMA valu_lead; each gap receives fillers up to its share of the issue cost."""
        ms = self.mfma
        nm = len(ms)
        gaps = max(nm, 1)
        # gap g follows MFMA g (g = 0 .. nm-1); gap -1 precedes the first MFMA
        sched = {g: [] for g in range(-1, gaps)}
        if self.other:
            og = max(1, int(round(gaps * other_frac)))
            tot = sum(c for c, _, _ in self.other)
            acc = 0.0
            for c, lines, _ in self.other:
                g = min(og - 1, int(acc / tot * og)) - 1
                sched[g].append(lines)
                acc += c
        if self.valu:
            first_gap = min(valu_lead, nm) - 1   # VALU from the gap after MFMA valu_lead-1 on
            vg = gaps - first_gap                # gaps first_gap .. nm-1
            tot = sum(c for c, _ in self.valu)
            acc = 0.0
            first = True
            for c, lines in self.valu:
                g = first_gap + min(vg - 1, int(acc / tot * vg))
                if first and lead_nop:
                    sched[g].append([f"s_nop {lead_nop}"])
                first = False
                sched[g].append(lines)
                acc += c
        for unit in sched[-1]:
            self._emit_unit(unit)
        for g, m in enumerate(ms):
            self._issue_mfma(m, kseqs, vseqs)
            for unit in sched[g]:
                self._emit_unit(unit)


def mask_scores(e, b):
    """SEG: if the current tile is a ragged segment tail, S_b of its keys past the segment's end
    -> -inf (rare path; the scores were just written by MFMAs: pad first)."""
    for j in range(2):
        lab = _label("m")
        e.op(f"s_cmp_eq_u32 %[tcur], %[trag{j}]")
        e.op(f"s_cbranch_scc0 {lab}")
        e.op("s_nop 15")
        for kb in range(2):
            for r in range(16):
                c = kb * 32 + (r & 3) + 8 * (r >> 2)  # key of S_b[16 kb + r] in the tile is c + 4 hi
                reg = vr(S[b] + 16 * kb + r)
                e.op(f"v_cmp_ge_i32 vcc, {c}, %[vk{j}]")
                e.op(f"v_cndmask_b32 {reg}, {reg}, %[ninf], vcc")
        e.op(f"{lab}:")


def body(t4, fill=False, drain=False, stage=True, vm=4):
    """Tile t with t % 4 == t4 (ring slot t4, register parity t4 & 1): K(t) in Kset[par] (read
    during X(t-1)), V(t-1) in Vset[par ^ 1]."""
    e = Emit()
    par, q = t4 & 1, (t4 & 1) ^ 1
    s_cur, s_next, s_stage = t4, (t4 + 1) & 3, (t4 + 3) & 3
    e.op(f"; ---- tile body t%4={t4} fill={int(fill)} drain={int(drain)} stage={int(stage)} vmcnt={vm}")
    # tile t+1 landed (tile t+2's pieces may stay in flight); every wave is done with slot t-1
    e.op(f"s_waitcnt vmcnt({min(vm + VM_SLACK, 63)})")
    if not NO_BARRIER:
        e.op("s_barrier")
    kseqs, vseqs = {}, {}
    if fill:
        # K(0) into Kset[0], then q-block 0's scores of tile 0
        p = Phase(e)
        p.read_k(par, s_cur, kseqs)
        p.qk(0, 0, par)
        p.qk(0, 1, par)
        p.emit(kseqs, vseqs, other_frac=0.01)
        e.wait_all_reads()
    if SEG:
        mask_scores(e, 0)  # S0(t): EXP0 runs in X
    # X(t): the LDS-DMA of tile t+3 first (its slot was freed by the barrier; the earlier it goes
    # out, the longer it has to land), then K(t+1)
    p = Phase(e)
    p.qk(1, 0, par)
    if not fill:
        p.pv(1, q)
    p.qk(1, 1, par)
    p.exp(0)
    if stage and DMA_IN_X:
        p.dma(s_stage)
    elif stage and DMA_SPLIT:
        p.dma(s_stage, range(DMA_SPLIT))
    if not drain:
        p.read_k(q, s_next, kseqs, (0,) if K1_IN_Y else (0, 1))
    if DMA_IN_X:
        p.emit(kseqs, vseqs, valu_lead=2 if fill else 1, lead_nop=15 if fill else 0, other_frac=0.5)
    else:
        p.read_v(par, s_cur, vseqs)
        p.emit(kseqs, vseqs, valu_lead=2 if fill else 1, lead_nop=15 if fill else X_LEAD_NOP, other_frac=X_READS)
    if SEG:
        mask_scores(e, 1)  # S1(t) (X's chains): EXP1 runs in Y
    # Y(t): V(t) early (P.V of q-block 0 starts after q.k^T's first chain)
    p = Phase(e)
    if not drain:
        p.qk(0, 0, q)
    p.pv(0, par)
    if not drain:
        p.qk(0, 1, q)
    p.exp(1)
    if K1_IN_Y and not drain:
        p.read_k(q, s_next, kseqs, (1,))
    if DMA_IN_X:
        p.read_v(par, s_cur, vseqs)
    elif stage:
        p.dma(s_stage, range(DMA_SPLIT, 4))
    # EXP1 reads S1 from X's last chain: two MFMAs and a pad first
    p.emit(kseqs, vseqs, valu_lead=2, lead_nop=7, other_frac=0.2 if DMA_IN_X else Y_DMA)
    if drain:
        # PV1(t): P1 was just written in place by EXP1 (VALU -> MFMA operand)
        e.op("s_nop 4")
        p = Phase(e)
        p.pv(1, par)
        p.emit(kseqs, vseqs)
    e.wait_all_reads()
    if SEG:
        e.op("s_add_u32 %[tcur], %[tcur], 1")
    return e.lines


def sweep():
    # tile 0 (fill, stages 3); groups of four staging tiles (t % 4 = 1, 2, 3, 0); the rem4 =
    # (ntiles - 4) % 4 remaining staging tiles; then the last three tiles (no stage; vmcnt 4 / 0 / 0;
    # the last one drains).  ntiles >= 4.
    L = lambda n: f"{n}_%="  # noqa: E731  (%= : a number unique to the asm statement instance)
    lines = body(0, fill=True)
    lines += [f"{L('Lgrp')}:", "s_cmp_eq_u32 %[n], 0", f"s_cbranch_scc1 {L('Lrem')}"]
    loop = body(1) + body(2) + body(3) + body(0)
    lines += loop
    lines += ["s_sub_u32 %[n], %[n], 1", f"s_branch {L('Lgrp')}", f"{L('Lrem')}:"]
    for r in range(4):
        lines += [f"s_cmp_eq_u32 %[rem], {r}", f"s_cbranch_scc1 {L(f'Lr{r}')}"]
    for r in range(4):
        lines += [f"{L(f'Lr{r}')}:"]
        for k in range(r):  # staging tiles t % 4 = 1 .. r
            lines += body(1 + k)
        t0 = 1 + r          # first tail tile (mod 4)
        lines += body(t0 & 3, stage=False, vm=4) + body((t0 + 1) & 3, stage=False, vm=0)
        lines += body((t0 + 2) & 3, drain=True, stage=False, vm=0)
        lines += [f"s_branch {L('Ldone')}"]
    lines += [f"{L('Ldone')}:"]
    # the compiler reads O / row sums right after the statement (XDL write -> read): pad
    lines += ["s_nop 15", "s_nop 15"]
    return lines, loop


def main():
    global SEG, VT
    out = ["// GENERATED by tools/gen_attn_pipe.py — do not edit by hand."]
    for seg, vt, name in ((False, False, "SR_ATTN_PIPE_ASM"), (True, False, "SR_ATTN_PIPE_ASM_SEG"),
                          (False, True, "SR_ATTN_PIPE_ASM_VT")):
        SEG, VT = seg, vt
        lines, loop = sweep()
        n_mfma = sum(1 for l in loop if l.startswith("v_mfma")) // 4
        n_valu = sum(1 for l in loop if l.startswith(("v_exp", "v_cvt"))) // 4
        n_ds = sum(1 for l in loop if l.startswith("ds_")) // 4
        n_all = sum(1 for l in loop if not l.startswith((";", "L")) and not l.endswith(":")) // 4
        out.append(f"// {name}: per tile {n_mfma} MFMA, {n_valu} exp/pack VALU, {n_ds} LDS fragment reads, "
                   f"{n_all} instructions (incl. the rare-path mask / switch blocks); {len(lines)} asm lines")
        out.append(f"#define {name} \\")
        out.append(" \\\n".join("  \"" + l + "\\n\\t\"" for l in lines))
        print(f"{name}: per tile {n_mfma} MFMA / {n_valu} VALU / {n_ds} ds reads / {n_all} instructions, "
              f"{len(lines)} asm lines")
    clob = ", ".join([f'"v{r}"' for r in NAMED_V] + [f'"a{r}"' for r in NAMED_A])
    out.append("#define SR_ATTN_PIPE_CLOBBERS " + clob)
    with open(OUT, "w") as f:
        f.write("\n".join(out) + "\n")


if __name__ == "__main__":
    main()
