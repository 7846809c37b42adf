#!/usr/bin/env python3
"""Generates self-supervise-sfm_amd/csrc/sr_attn_pipe.inc: the hand-scheduled steady-state sweep
of attn_bf16_kernel<4, 2, KIND, PIPE=true> (sr_attn.hip) as ONE inline-asm statement.

Why asm: the pipelined sweep pairs one q-block's q.k^T MFMAs with the other q-block's exp2 / pack
stretch inside each wave (DESIGN.md "Attention"); compiled from C++ it needs ~270 VGPRs at two
waves per SIMD and spills (185 VGPRs), or runs one wave per SIMD at half speed.  Here the score /
P registers are named (v160-v253, in place: P overwrites the scores it came from) and everything
else (O, Q fragments, row sums, addresses) stays a compiler-allocated operand.

Per tile t (steady state; q-block 0's scores S0 of tile t were produced by the previous tile's Y):
  [wait tile t+1 (vmcnt), s_barrier, LDS-DMA of tile t+3 into slot (t+3) mod 5]
  X(t): MFMA  QK1 kb0 chain (S1[0:15]) | PV1(t-1) (P1 in S1[16:31], V of tile t-1) | QK1 kb1 chain
        VALU  EXP0(t): S0 -> P0, written in place into S0[16:31]
  Y(t): MFMA  QK0(t+1) kb0 chain (S0[0:15]) | PV0(t) (P0 in S0[16:31], V of tile t) | QK0(t+1) kb1
        VALU  EXP1(t): S1 -> P1 in place into S1[16:31]
EXP order per q-block: (kb, s2) = (1,0), (1,1), (0,0), (0,1); P fragment idx i at S[16+4i : 19+4i].
Fill (tile 0): QK0(0) both chains before X, no PV1 in X.  Drain (last tile): no QK0(t+1) in Y,
then PV1(t).  The statement runs a wave's whole sweep over ntiles >= 4 full tiles of one key
segment; the last three tiles stage nothing.  Hazards handled here: lgkmcnt counted per fragment read (LDS returns in order),
>= 3 fragment buffers per kind (a buffer is rewritten one MFMA after its reader issued), s_nop
after the MFMA chain whose scores the next VALU phase reads, M0 -> LDS-DMA s_nop 0.

    python3 tools/gen_attn_pipe.py          (writes the .inc; committed, regenerate after edits)
"""

import os

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "..", "self-supervise-sfm_amd", "csrc", "sr_attn_pipe.inc")

# named registers
S = {0: 160, 1: 192}          # S_b: 32 VGPRs, kb block k at S_b + 16k
KF = [224, 228, 232]          # K fragment buffers (4 VGPRs each)
VF = [236, 240, 244]          # V^T fragment buffers (2 tr reads = 4 VGPRs each)
KA = 248                      # K fragment address (s = 0) of the tile in use
VA = 249                      # V fragment address (db = 0) of the tile in use
AT = 250                      # address temporary: KA ^ 32 s, VA ^ 64 (db = 1)
NAMED = list(range(160, 251))
# the lane offsets satisfy koff[s] = koff[0] ^ 32 s and voff1 = voff0 ^ 64 (the XOR swizzles of
# sr_attn.hip), and slot + lds0 is a multiple of 128 (checked by the caller), so one address
# register per operand serves every fragment
# scalar scratch: slot offsets are derived into these
EXP_ORDER = [(1, 0), (1, 1), (0, 0), (0, 1)]  # (kb, s2) in EXP / P-fragment order
TILE_B = 8192                 # bytes of a K (or V) tile; V sits after K in a stage
STAGE_B = 2 * TILE_B
RING = 5 * STAGE_B


def vr(a, n=1):
    return f"v{a}" if n == 1 else f"v[{a}:{a + n - 1}]"


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
        if seq <= self.waited:
            return
        n = self.reads - seq - 1
        self.op(f"s_waitcnt lgkmcnt({min(n, 15)})")
        self.waited = seq

    def wait_all_reads(self):
        if self.waited < self.reads - 1:
            self.op("s_waitcnt lgkmcnt(0)")
            self.waited = self.reads - 1


def slot_derive(e, dst, k):
    """dst = slot offset of tile t+k (k in 1..4) from %[slot] (tile t): (slot + k*STAGE_B) wrapped
    into the 5-stage ring (the ring base %[lds0] is added by the caller)."""
    e.op(f"s_add_u32 {dst}, %[slot], {k * STAGE_B}")
    e.op(f"s_sub_u32 %[stmp], {dst}, {RING}")
    e.op(f"s_cmp_ge_u32 {dst}, {RING}")
    e.op(f"s_cselect_b32 {dst}, %[stmp], {dst}")


def k_addresses(e, sreg):
    """KA = lds0 + slot (sreg) + koff[0]"""
    e.op(f"v_add_u32 {vr(KA)}, {sreg}, %[koff0]")


def v_addresses(e, sreg):
    """VA = lds0 + slot (sreg) + voff[0] (+ TILE_B as the instruction offset)"""
    e.op(f"v_add_u32 {vr(VA)}, {sreg}, %[voff0]")


class Phase:
    """One X or Y phase: an ordered MFMA list (each with the fragment it reads) interleaved with
    an ordered VALU list; fragments are prefetched two MFMAs ahead into rotating buffers."""

    def __init__(self, e):
        self.e = e
        self.mfma = []   # (kind, params)
        self.valu = []   # text
        self.kbuf = 0
        self.vbuf = 0

    def qk(self, b, kb):
        for s in range(4):
            self.mfma.append(("qk", (b, kb, s)))

    def pv(self, b):
        for i, (kb, s2) in enumerate(EXP_ORDER):
            self.mfma.append(("rs", (b, i)))
            for db in range(2):
                self.mfma.append(("pv", (b, i, kb, s2, db)))

    def exp(self, b):
        base = S[b]
        for i, (kb, s2) in enumerate(EXP_ORDER):
            src = base + 16 * kb + 8 * s2
            for j in range(8):
                self.valu.append(f"v_exp_f32 {vr(src + j)}, {vr(src + j)}")
            dst = base + 16 + 4 * i
            for jj in range(4):
                self.valu.append(f"v_cvt_pk_bf16_f32 {vr(dst + jj)}, {vr(src + 2 * jj)}, {vr(src + 2 * jj + 1)}")

    def _load(self, m):
        kind, p = m
        e = self.e
        if kind == "qk":
            b, kb, s = p
            buf = KF[self.kbuf % len(KF)]
            self.kbuf += 1
            if s:
                e.op(f"v_xor_b32 {vr(AT)}, {32 * s}, {vr(KA)}")
            seq = e.ds(f"ds_read_b128 {vr(buf, 4)}, {vr(AT if s else KA)} offset:{kb * 4096}")
            return (buf, seq)
        if kind == "pv":
            b, i, kb, s2, db = p
            buf = VF[self.vbuf % len(VF)]
            self.vbuf += 1
            off = TILE_B + (kb * 32 + 16 * s2) * 128
            if db:
                e.op(f"v_xor_b32 {vr(AT)}, 64, {vr(VA)}")
            a = vr(AT if db else VA)
            e.ds(f"ds_read_b64_tr_b16 {vr(buf, 2)}, {a} offset:{off}")
            seq = e.ds(f"ds_read_b64_tr_b16 {vr(buf + 2, 2)}, {a} offset:{off + 1024}")
            return (buf, seq)
        return (None, None)

    def _issue(self, m, frag):
        kind, p = m
        e = self.e
        if kind == "qk":
            b, kb, s = p
            buf, seq = frag
            e.wait_read(seq)
            acc = vr(S[b] + 16 * kb, 16)
            c = "0" if s == 0 else acc
            e.op(f"v_mfma_f32_32x32x16_bf16 {acc}, {vr(buf, 4)}, %[q{b}{s}], {c}")
        elif kind == "rs":
            b, i = p
            e.op(f"v_mfma_f32_16x16x32_bf16 %[l{b}], %[suma], {vr(S[b] + 16 + 4 * i, 4)}, %[l{b}]")
        else:
            b, i, kb, s2, db = p
            buf, seq = frag
            e.wait_read(seq)
            e.op(f"v_mfma_f32_32x32x16_bf16 %[o{b}{db}], {vr(buf, 4)}, {vr(S[b] + 16 + 4 * i, 4)}, %[o{b}{db}]")

    def emit(self, valu_lead=0, lead_nop=0):
        """valu_lead: MFMAs issued before the first VALU (the scores the VALU reads must come from
        MFMAs that completed); lead_nop: s_nop count placed before the first VALU.  The VALU list
        is spread evenly over the gaps after MFMA valu_lead-1 .. the last MFMA."""
        e = self.e
        ms, vs = self.mfma, self.valu
        nm, nv = len(ms), len(vs)
        frags = [None] * nm
        ahead = 2
        for j in range(min(ahead, nm)):
            frags[j] = self._load(ms[j])
        lead = min(valu_lead, nm)
        slots = nm - lead + 1 if nm > 0 else 1
        vi = 0
        nop_done = False

        def flush(target):
            nonlocal vi, nop_done
            if target > vi and lead_nop and not nop_done:
                e.op(f"s_nop {lead_nop}")
                nop_done = True
            while vi < target:
                e.op(vs[vi])
                vi += 1

        if lead == 0:
            flush(-(-nv // slots))
        for i, m in enumerate(ms):
            if i + ahead < nm:
                frags[i + ahead] = self._load(ms[i + ahead])
            self._issue(m, frags[i])
            k = i + 2 - lead  # gaps filled so far (1 .. slots - 1 + ...)
            if k >= 1:
                flush(min(nv, -(-nv * (k + (1 if lead == 0 else 0)) // slots)))
        flush(nv)


def body(fill, drain, stage, vm):
    e = Emit()
    e.op(f"; ---- tile body fill={fill} drain={drain} stage={stage} vmcnt={vm}")
    # tile t+1 landed (tile t+2's pieces may stay in flight), everyone done with slot t-2
    e.op(f"s_waitcnt vmcnt({vm})")
    e.op("s_barrier")
    if stage:
        # LDS-DMA of tile t+3 (4 pieces of 8 rows per wave) into slot (t+3) mod 5
        slot_derive(e, "%[sst]", 3)
        e.op("s_add_u32 %[sst], %[sst], %[ldsv]")
        for i in range(4):
            e.op(f"s_add_u32 m0, %[sst], {i * 1024}")
            e.op("s_nop 0")
            e.op(f"global_load_lds_dwordx4 %[dma{i & 1}], %[{'sp' if i < 2 else 'sp2'}]")
        for i in range(2):
            e.op(f"v_add_u32 %[dma{i}], %[sstep], %[dma{i}]")
    # addresses: K of tile t (X), V of tile t-1 (X)
    e.op("s_add_u32 %[sk], %[slot], %[lds0]")
    k_addresses(e, "%[sk]")
    slot_derive(e, "%[sv]", 4)  # t + 4 = t - 1 (mod 5)
    e.op("s_add_u32 %[sv], %[sv], %[lds0]")
    v_addresses(e, "%[sv]")
    if fill:
        p = Phase(e)
        p.qk(0, 0)
        p.qk(0, 1)
        p.emit()
    # X(t)
    p = Phase(e)
    p.qk(1, 0)
    if not fill:
        p.pv(1)
    p.qk(1, 1)
    p.exp(0)
    # fill: S0 was just written by the chain above -> keep the first VALU behind 2 MFMAs + nops
    p.emit(valu_lead=2 if fill else 1, lead_nop=15 if fill else 0)
    # Y(t): V of tile t, K of tile t+1
    e.op("s_add_u32 %[sv], %[slot], %[lds0]")
    v_addresses(e, "%[sv]")
    if not drain:
        slot_derive(e, "%[sk]", 1)
        e.op("s_add_u32 %[sk], %[sk], %[lds0]")
        k_addresses(e, "%[sk]")
    p = Phase(e)
    if not drain:
        p.qk(0, 0)
    p.pv(0)
    if not drain:
        p.qk(0, 1)
    p.exp(1)
    # EXP1 reads S1[16:31] from X's last chain: two MFMAs and 15 wait states first
    p.emit(valu_lead=2, lead_nop=15)
    if drain:
        # PV1(t): P1 was just written in place by EXP1 (VALU -> MFMA B operand: 2 wait states)
        e.op("s_nop 4")
        p = Phase(e)
        p.pv(1)
        p.emit()
    e.wait_all_reads()
    # next tile: slot += 1 (mod 5)
    slot_derive(e, "%[slot]", 1)
    return e.lines


def main():
    # the whole sweep of a wave: tile 0 (fill, stages tile 3), tiles 1 .. ntiles-4 (loop, stage t+3),
    # then the last three tiles (no stage; vmcnt 4 / 0 / 0; the last one drains).  ntiles >= 4.
    first = body(1, 0, 1, 4)
    loop = body(0, 0, 1, 4)
    tail = body(0, 0, 0, 4) + body(0, 0, 0, 0) + body(0, 1, 0, 0)
    L = lambda n: f"{n}_%="  # noqa: E731  (%= : a number unique to the asm statement instance)
    lines = first
    lines.append(f"{L('Lloop')}:")
    lines.append("s_cmp_eq_u32 %[n], 0")
    lines.append(f"s_cbranch_scc1 {L('Ltail')}")
    lines += loop
    lines.append("s_sub_u32 %[n], %[n], 1")
    lines.append(f"s_branch {L('Lloop')}")
    lines.append(f"{L('Ltail')}:")
    lines += tail
    # the compiler reads O / row sums right after the statement (XDL write -> VALU read): pad the
    # last MFMAs out (16-pass worst case, cdna_hip_programming.md hazard table)
    lines += ["s_nop 15", "s_nop 15"]
    text = " \\\n".join("  \"" + l + "\\n\\t\"" for l in lines)
    clob = ", ".join(f'"v{r}"' for r in NAMED)
    n_mfma = sum(1 for l in loop if l.startswith("v_mfma"))
    n_valu = sum(1 for l in loop if l.startswith(("v_exp", "v_cvt")))
    n_ds = sum(1 for l in loop if l.startswith("ds_"))
    with open(OUT, "w") as f:
        f.write("// GENERATED by tools/gen_attn_pipe.py — do not edit by hand.\n")
        f.write(f"// steady-state tile: {n_mfma} MFMA, {n_valu} exp/pack VALU, {n_ds} LDS fragment reads,\n")
        f.write(f"// {len(loop)} lines; {len(lines)} lines in all\n")
        f.write("#define SR_ATTN_PIPE_ASM \\\n")
        f.write(text + "\n")
        f.write("#define SR_ATTN_PIPE_CLOBBERS " + clob + "\n")
    print(f"wrote {OUT}: steady tile {n_mfma} MFMA / {n_valu} VALU / {n_ds} ds reads, {len(lines)} asm lines")


if __name__ == "__main__":
    main()
