#!/usr/bin/env python
"""Kernel microbenchmarks at the N=32 @ 518 hot-path shapes (random data).

    python tools/kbench.py [attn] [gemm] [ln]

Each case: warm up, then time R launches with HIP events on the launching stream;
prints TFLOP/s (MFMA-bound kernels) or GB/s (LayerNorm) and the fraction of peak.
"""

import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "self-supervise-sfm_amd"))

import torch  # noqa: E402

from sailrecon_amd import _lib, ops  # noqa: E402

DEV = "cuda"
PEAK = 2500.0


def timeit(fn, reps=10, warm=2):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def attn():
    C, H, D = 1024, 16, 64
    P, N = 1374, 32
    cases = {
        "global L=43968": dict(rows=N * P, batch=1, lq=N * P, l0=N * P, kb=0),
        "frame 64x1374": dict(rows=2 * N * P, batch=2 * N, lq=P, l0=P, kb=P),
    }
    # SR_KB_STATIC=1: pass the keys' true max norm as the static bound (runtime.key_norm_bound's
    # role for qk-norm blocks) instead of the key scan
    static = os.environ.get("SR_KB_STATIC", "0") == "1"
    # SR_KB_TAIL=1 (default): buffers with 64 readable rows after them, as the aggregator's
    # workspace (ops.attention tail_readable: ragged / two-segment launches may take the asm sweep)
    tail = os.environ.get("SR_KB_TAIL", "1") == "1"
    pad = 64 if tail else 0
    for name, c in cases.items():
        qkv = torch.randn(c["rows"] + pad, 3 * C, device=DEV, dtype=torch.bfloat16)[:c["rows"]]
        o = torch.empty(c["rows"], C, device=DEV, dtype=torch.bfloat16)
        kb = float(qkv[:, C:2 * C].float().view(-1, H, D).norm(dim=-1).max()) if static else 0.0

        def f():
            ops.attention(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], o, heads=H, head_dim=D, batch=c["batch"],
                          lq=c["lq"], q_bstride=c["lq"], l0=c["l0"], k0_bstride=c["kb"], key_norm_max=kb,
                          tail_readable=tail)
        ms = timeit(f, reps=5 if c["batch"] == 1 else 10)
        fl = 4.0 * c["batch"] * H * c["lq"] * c["l0"] * D
        print(f"attn {name:18s} {ms:8.3f} ms  {fl / ms / 1e9:8.1f} TF/s  {fl / ms / 1e9 / PEAK:6.1%}")
    # reloc: 32 query frames x (32*305 subsample + own 1374)
    nsub = N * 305
    qkv = torch.randn(N * P + pad, 3 * C, device=DEV, dtype=torch.bfloat16)[:N * P]
    kv = torch.randn(nsub + pad, 2 * C, device=DEV, dtype=torch.bfloat16)[:nsub]
    o = torch.empty(N * P, C, device=DEV, dtype=torch.bfloat16)
    kb = max(float(qkv[:, C:2 * C].float().view(-1, H, D).norm(dim=-1).max()),
             float(kv[:, :C].float().view(-1, H, D).norm(dim=-1).max())) if static else 0.0

    def f():
        ops.attention(qkv[:, :C], kv[:, :C], kv[:, C:], o, heads=H, head_dim=D, batch=N, lq=P, q_bstride=P, l0=nsub,
                      k0_bstride=0, k1=qkv[:, C:2 * C], v1=qkv[:, 2 * C:], l1=P, k1_bstride=P, key_norm_max=kb,
                      tail_readable=tail)
    ms = timeit(f)
    fl = 4.0 * N * H * P * (nsub + P) * D
    print(f"attn {'reloc 32x(9760+1374)':18s} {ms:8.3f} ms  {fl / ms / 1e9:8.1f} TF/s  {fl / ms / 1e9 / PEAK:6.1%}")
    # the same reloc attention split (aggregator SR_RELOC_SPLIT=1): all 43,968 query rows against the
    # subsample's 152 whole tiles (one long query set), each frame against the last 32 subsample
    # keys + itself, LSE merge
    rows, nf = N * P, nsub // 64 * 64
    o_parts, lse_parts = ops.key_split_workspace(DEV, 2, rows, C, H, name="kb_reloc_split")

    def pa():
        ops.attention(qkv[:, :C], kv[:nf, :C], kv[:nf, C:], o_parts[:rows], heads=H, head_dim=D, batch=1, lq=rows,
                      q_bstride=0, l0=nf, k0_bstride=0, key_norm_max=kb, lse=lse_parts[0].view(-1), tail_readable=tail)

    def pb():
        ops.attention(qkv[:, :C], kv[nf:, :C], kv[nf:, C:], o_parts[rows:], heads=H, head_dim=D, batch=N, lq=P,
                      q_bstride=P, l0=nsub - nf, k0_bstride=0, k1=qkv[:, C:2 * C], v1=qkv[:, 2 * C:], l1=P,
                      k1_bstride=P, key_norm_max=kb, lse=lse_parts[1].view(-1), tail_readable=tail)

    def pm():
        ops.attn_merge_n(o_parts, lse_parts, o, parts=2, rows=rows, heads=H, head_dim=D, seg_rows=[rows, P])

    def pbm():  # the aggregator's form: the second pass merges the first in its epilogue
        ops.attention(qkv[:, :C], kv[nf:, :C], kv[nf:, C:], o, heads=H, head_dim=D, batch=N, lq=P,
                      q_bstride=P, l0=nsub - nf, k0_bstride=0, k1=qkv[:, C:2 * C], v1=qkv[:, 2 * C:], l1=P,
                      k1_bstride=P, key_norm_max=kb, tail_readable=tail, merge_o=o_parts[:rows],
                      merge_lse=lse_parts[0])
    ta, tb, tm, tbm = timeit(pa), timeit(pb), timeit(pm), timeit(pbm)
    print(f"attn reloc split: subsample pass {ta:.3f} ms ({4.0 * H * rows * nf * D / ta / 1e9:.1f} TF/s), "
          f"tail+own pass {tb:.3f} ms, merge {tm:.3f} ms, total {ta + tb + tm:.3f} ms  "
          f"{fl / (ta + tb + tm) / 1e9:8.1f} TF/s; merge-in pass {tbm:.3f} ms, total {ta + tbm:.3f} ms  "
          f"{fl / (ta + tbm) / 1e9:8.1f} TF/s")


def attn_pair():
    """C3 global attention + the split reloc's subsample pass: apart vs one sr_attention_pair launch."""
    C, H, D, P, N = 1024, 16, 64, 1374, 32
    L, nf = N * P, N * 305 // 64 * 64
    qkv = torch.randn(L + 64, 3 * C, device=DEV, dtype=torch.bfloat16)[:L]
    qr = torch.randn(L, C, device=DEV, dtype=torch.bfloat16)
    kv = torch.randn(nf, 2 * C, device=DEV, dtype=torch.bfloat16)
    og, oa = (torch.empty(L, C, device=DEV, dtype=torch.bfloat16) for _ in range(2))
    lse = torch.empty(H, L, device=DEV)
    kb = lambda k: 1.01 * float(k.float().view(-1, H, D).norm(dim=-1).max())  # noqa: E731
    kbg, kbr = kb(qkv[:, C:2 * C]), kb(kv[:, :C])

    def apart():
        ops.attention(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], og, heads=H, head_dim=D, batch=1, lq=L,
                      q_bstride=0, l0=L, k0_bstride=0, key_norm_max=kbg)
        ops.attention(qr, kv[:, :C], kv[:, C:], oa, heads=H, head_dim=D, batch=1, lq=L, q_bstride=0, l0=nf,
                      k0_bstride=0, key_norm_max=kbr, lse=lse.view(-1))

    def paired():
        ops.attention_pair(dict(q=qkv[:, :C], k0=qkv[:, C:2 * C], v0=qkv[:, 2 * C:], o=og, lq=L, l0=L, key_norm_max=kbg),
                           dict(q=qr, k0=kv[:, :C], v0=kv[:, C:], o=oa, lq=L, l0=nf, key_norm_max=kbr,
                                lse=lse.view(-1)), heads=H, head_dim=D)
    vtg = torch.empty(ops.vt_tile_shape(L, H), device=DEV, dtype=torch.bfloat16)
    vtr = torch.empty(ops.vt_tile_shape(nf, H), device=DEV, dtype=torch.bfloat16)

    def tiles():
        ops.vt_tiles(qkv[:, 2 * C:], L, H, vtg)
        ops.vt_tiles(kv[:, C:], nf, H, vtr)

    def paired_vt():
        ops.attention_pair(dict(q=qkv[:, :C], k0=qkv[:, C:2 * C], v0=qkv[:, 2 * C:], o=og, lq=L, l0=L, key_norm_max=kbg,
                                vt=vtg),
                           dict(q=qr, k0=kv[:, :C], v0=kv[:, C:], o=oa, lq=L, l0=nf, key_norm_max=kbr,
                                lse=lse.view(-1), vt=vtr), heads=H, head_dim=D)
    tiles()
    fl = 4.0 * H * L * (L + nf) * D
    for i in range(2):
        ta, tp, tv, tt = (timeit(apart, reps=5), timeit(paired, reps=5), timeit(paired_vt, reps=5),
                          timeit(tiles, reps=20))
        print(f"attn pair C3 global + reloc subsample: apart {ta:.3f} ms ({fl / ta / 1e9:.1f} TF/s), "
              f"paired {tp:.3f} ms ({fl / tp / 1e9:.1f} TF/s), paired V^T {tv:.3f} ms ({fl / tv / 1e9:.1f} TF/s) "
              f"+ its two sr_vt_tiles {tt * 1e3:.1f} us", flush=True)


def qk_normed(rows, g, gen, H=16, D=64):
    """[rows, H*D] bf16 as the aggregator's qk-norm produces it (attention.py:49-50,78): per-head
    LayerNorm of a gaussian times w + b, w = g (1 + 0.02 n), b = 0.02 n (the synthetic rule's LN
    affine scaled by the qk-gain g; trained q_norm / k_norm gains sit around 2-3).  Returns the
    tensor and runtime.key_norm_bound's static bound sqrt(D) max|w| + |b| (x 1 + 2^-6)."""
    x = torch.randn(rows, H, D, device=DEV, generator=gen)
    x = (x - x.mean(-1, keepdim=True)) / x.std(-1, keepdim=True, unbiased=False)
    w = g * (1.0 + 0.02 * torch.randn(D, device=DEV, generator=gen))
    b = 0.02 * torch.randn(D, device=DEV, generator=gen)
    kb = (D ** 0.5 * float(w.abs().max()) + float(b.norm())) * (1.0 + 2.0 ** -6)
    return (x * w + b).reshape(rows, H * D).bfloat16(), kb


def attn_gain():
    """the hand-scheduled global sweep at qk-norm gains g = 1, 2, 4 (the bound
    qb grows as g^2).  Global L = 43,968 alone and paired with the reloc subsample pass, with the
    waves that ran the asm sweep / the compiled loop (sr_attn_desc.sweep_stats)."""
    C, H, D, P, N = 1024, 16, 64, 1374, 32
    L, nf = N * P, N * 305 // 64 * 64
    fl1 = 4.0 * H * L * L * D
    fl2 = 4.0 * H * L * (L + nf) * D
    gains = [float(x) for x in os.environ.get("SR_QK_GAINS", "1,2,3,4").split(",")]
    for g in gains:
        gen = torch.Generator(device=DEV).manual_seed(1)
        q, _ = qk_normed(L, g, gen)
        k, kb = qk_normed(L, g, gen)
        v = torch.randn(L, C, device=DEV, dtype=torch.bfloat16)
        qr, _ = qk_normed(L, g, gen)
        ks, kbs = qk_normed(nf, g, gen)
        vs = torch.randn(nf, C, device=DEV, dtype=torch.bfloat16)
        o, orr = torch.empty_like(q), torch.empty_like(q)
        lse = torch.empty(H, L, device=DEV)
        st = torch.zeros(2, dtype=torch.int32, device=DEV)

        def glob(stats=None):
            ops.attention(q, k, v, o, heads=H, head_dim=D, batch=1, lq=L, q_bstride=0, l0=L, k0_bstride=0,
                          key_norm_max=kb, sweep_stats=stats)

        def pair(stats=None):
            ops.attention_pair(dict(q=q, k0=k, v0=v, o=o, lq=L, l0=L, key_norm_max=kb, sweep_stats=stats),
                               dict(q=qr, k0=ks, v0=vs, o=orr, lq=L, l0=nf, key_norm_max=kbs, lse=lse.view(-1),
                                    sweep_stats=stats), heads=H, head_dim=D)
        glob(st)
        torch.cuda.synchronize()
        sg = st.tolist()
        st.zero_()
        pair(st)
        torch.cuda.synchronize()
        sp = st.tolist()
        tg, tp = timeit(glob, reps=5), timeit(pair, reps=5)
        qb = 1.4426950408889634 / 8 * kb * kb
        print(f"attn qk-gain {g:.1f} (bound qb ~ {qb:6.1f}): global {tg:.3f} ms ({fl1 / tg / 1e9:.1f} TF/s, asm waves "
              f"{sg[0]}/{sg[0] + sg[1]}); pair {tp:.3f} ms ({fl2 / tp / 1e9:.1f} TF/s, asm waves {sp[0]}/{sp[0] + sp[1]})",
              flush=True)
        # frame / DINO attention (64 frames x 1374, compiled two-workgroups-per-CU sweep) at the same gain
        S = 64
        qf = torch.cat([q, qr])[:S * P] if 2 * L >= S * P else None
        kf, kbf = qk_normed(S * P, g, gen)
        vf = torch.randn(S * P, C, device=DEV, dtype=torch.bfloat16)
        of = torch.empty_like(vf)
        tf = timeit(lambda: ops.attention(qf, kf, vf, of, heads=H, head_dim=D, batch=S, lq=P, q_bstride=P, l0=P,
                                          k0_bstride=P, key_norm_max=kbf), reps=10)
        ff = 4.0 * S * H * P * P * D
        print(f"attn qk-gain {g:.1f} frame 64x1374: {tf:.3f} ms ({ff / tf / 1e9:.1f} TF/s)", flush=True)


def attn_frame_cfg():
    """Frame / DINO attention (64 frames x 1374 tokens, static key bound) under each bf16 workgroup
    shape (SR_ATTN_CFG: 0 = 4 waves x 2 q-blocks, 1 = 8 x 1, 2 = 2 x 2 = 128 rows), interleaved."""
    C, H, D, P, S = 1024, 16, 64, 1374, 64
    qkv = torch.randn(S * P + 64, 3 * C, device=DEV, dtype=torch.bfloat16)[:S * P]
    o = torch.empty(S * P, C, device=DEV, dtype=torch.bfloat16)
    kb = float(qkv[:, C:2 * C].float().view(-1, H, D).norm(dim=-1).max())
    fl = 4.0 * S * H * P * P * D
    for cfg in (0, 1, 2, 0, 1, 2):
        with ops.tuning(SR_ATTN_CFG=cfg):
            ms = timeit(lambda: ops.attention(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], o, heads=H, head_dim=D,
                                              batch=S, lq=P, q_bstride=P, l0=P, k0_bstride=P, key_norm_max=kb,
                                              tail_readable=True), reps=20)
            kern = ops.last_kernel()
        print(f"attn frame cfg {cfg} ({kern}): {ms:.3f} ms  {fl / ms / 1e9:.1f} TF/s", flush=True)


def attn_frame_diag():
    """Where the frame attention loses against the long sweep: the same launch with no ragged
    q-tile (lq = 1280 = 5 x 256), with full key tiles (l0 = 1408), and with 4x longer key sweeps
    (l0 = 5496, the neighbouring frames' keys), 16 heads, static key bound."""
    C, H, D, P = 1024, 16, 64, 1374
    B = 64
    qkv = torch.randn(B * P + 8 * P, 3 * C, device=DEV, dtype=torch.bfloat16)
    o = torch.empty(B * P, C, device=DEV, dtype=torch.bfloat16)
    kb = 1.01 * float(qkv[:, C:2 * C].float().view(-1, H, D).norm(dim=-1).max())
    warm = torch.randn(8192, 8192, device=DEV, dtype=torch.bfloat16)
    for _ in range(20):  # clocks up before the first timed case
        warm @ warm
    for lq, l0, b in ((P, P, B), (1280, P, B), (P, 1408, B), (1280, 1408, B), (1280, 4 * P, B),
                      (P, 4 * P, B), (1024, P, B), (768, P, B), (512, P, B), (256, P, B)):
        def f():
            ops.attention(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], o, heads=H, head_dim=D, batch=b, lq=lq,
                          q_bstride=P, l0=l0, k0_bstride=P, key_norm_max=kb, tail_readable=True)
        ms = timeit(f)
        fl = 4.0 * b * H * lq * l0 * D
        print(f"attn frame-diag b={b} lq={lq:5d} l0={l0:5d} {ms:8.3f} ms  {fl / ms / 1e9:8.1f} TF/s", flush=True)


def attn_rank():
    """Per-rank global attention of the frame-sharded C3 forward: 32/G anchors' queries against
    all 43,968 anchor keys (one pass), G = 2, 4, 8."""
    C, H, D, P, N = 1024, 16, 64, 1374, 32
    L = N * P
    qkv = torch.randn(L, 3 * C, device=DEV, dtype=torch.bfloat16)
    kb = float(qkv[:, C:2 * C].float().view(-1, H, D).norm(dim=-1).max())
    for G in (1, 2, 4, 8):
        lq = L // G
        o = torch.empty(lq, C, device=DEV, dtype=torch.bfloat16)

        def f():
            ops.attention(qkv[:lq, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], o, heads=H, head_dim=D, batch=1, lq=lq,
                          q_bstride=0, l0=L, k0_bstride=0, key_norm_max=kb)
        saved = ops._KSPLIT_ENV
        for split in ("0", "auto", "2", "3", "4", "6", "8"):
            ops._KSPLIT_ENV = None if split == "auto" else split
            parts = ops.key_split_parts(dtype=torch.bfloat16, batch=1, lq=lq, heads=H, l0=L, l1=0, mask_mode=0)
            ms = timeit(f, reps=5)
            fl = 4.0 * H * lq * L * D
            print(f"attn rank G={G} lq={lq:6d} keys={L} split={split:4s}(S={parts}) {ms:8.3f} ms  "
                  f"{fl / ms / 1e9:8.1f} TF/s  {fl / ms / 1e9 / PEAK:6.1%}")
        ops._KSPLIT_ENV = saved


def attn_rank_seg():
    """attn_rank's key-split launches (auto S) with the chunks' tails readable: the compiled sweep
    vs the hand-scheduled _SEG sweep (SR_ATTN_PIPE_SEG=1), which masks each chunk's ragged last
    key tile (43,968 / S keys are not whole 64-key tiles for S = 2, 4, 8)."""
    C, H, D, P, N = 1024, 16, 64, 1374, 32
    L = N * P
    qkv = torch.randn(L + 64, 3 * C, device=DEV, dtype=torch.bfloat16)[:L]
    kb = float(qkv[:, C:2 * C].float().view(-1, H, D).norm(dim=-1).max())
    for G in (2, 4, 8):
        lq = L // G
        S = ops.key_split_parts(dtype=torch.bfloat16, batch=1, lq=lq, heads=H, l0=L, l1=0, mask_mode=0)
        o_parts, lse_parts = ops.key_split_workspace(qkv.device, S, lq, C, H)
        chunk = L // S
        d = ops._attn_desc(qkv[:lq, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], o_parts, heads=H, head_dim=D, batch=S,
                           lq=lq, q_bstride=0, l0=chunk, k0_bstride=chunk, lse=lse_parts)
        d.o_bstride = lq
        d.key_norm_max = kb
        d.tail_rows_readable = 64
        fl = 4.0 * H * lq * L * D

        def f():
            ops.check(_lib.load().sr_attention(ops._stream(qkv), ops.dtype_code(qkv.dtype), ops.ctypes.byref(d)),
                      "sr_attention")
        res = {}
        for seg in ("0", "1", "0", "1"):
            ops.set_tuning("SR_ATTN_PIPE_SEG", int(seg))
            ms = timeit(f, reps=10)
            res.setdefault(seg, []).append(ms)
        outs = []
        for seg in ("0", "1"):
            ops.set_tuning("SR_ATTN_PIPE_SEG", int(seg))
            o_parts.zero_()
            f()
            torch.cuda.synchronize()
            outs.append((o_parts[:S * lq].float().clone(), lse_parts.clone()))
        ops.set_tuning("SR_ATTN_PIPE_SEG", 0)
        print(f"attn rank seg G={G} max |o| diff {float((outs[0][0] - outs[1][0]).abs().max()):.3e} "
              f"max |lse| diff {float((outs[0][1] - outs[1][1]).abs().max()):.3e}")
        for seg, v in res.items():
            print(f"attn rank seg G={G} S={S} chunk={chunk} pipe_seg={seg} "
                  + " ".join(f"{m:7.3f} ms ({fl / m / 1e9:7.1f} TF/s)" for m in v))


def attn_rank_small():
    """Per-rank reloc (32/G query frames x [9760 shared subsample + own 1374]) and frame
    (64/G frames x 1374) attention of the frame-sharded C3 forward, G = 1, 2, 4, 8."""
    C, H, D, P, N = 1024, 16, 64, 1374, 32
    nsub = N * 305
    for G in (1, 2, 4, 8):
        nq = N // G
        qkv = torch.randn(2 * nq * P, 3 * C, device=DEV, dtype=torch.bfloat16)
        kv = torch.randn(nsub, 2 * C, device=DEV, dtype=torch.bfloat16)
        o = torch.empty(2 * nq * P, C, device=DEV, dtype=torch.bfloat16)
        kb = 1.01 * max(float(qkv[:, C:2 * C].float().view(-1, H, D).norm(dim=-1).max()),
                        float(kv[:, :C].float().view(-1, H, D).norm(dim=-1).max()))

        def rl():
            ops.attention(qkv[:nq * P, :C], kv[:, :C], kv[:, C:], o, heads=H, head_dim=D, batch=nq, lq=P,
                          q_bstride=P, l0=nsub, k0_bstride=0, k1=qkv[:nq * P, C:2 * C], v1=qkv[:nq * P, 2 * C:],
                          l1=P, k1_bstride=P, key_norm_max=kb)

        def fr():
            ops.attention(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], o, heads=H, head_dim=D, batch=2 * nq, lq=P,
                          q_bstride=P, l0=P, k0_bstride=P, key_norm_max=kb)
        ms = timeit(rl)
        fl = 4.0 * nq * H * P * (nsub + P) * D
        print(f"attn rank G={G} reloc {nq:2d}x({nsub}+{P}) {ms:8.3f} ms  {fl / ms / 1e9:8.1f} TF/s")
        ms = timeit(fr)
        fl = 4.0 * 2 * nq * H * P * P * D
        print(f"attn rank G={G} frame {2 * nq:2d}x{P}        {ms:8.3f} ms  {fl / ms / 1e9:8.1f} TF/s")


def attn_rank_cfg():
    """attn_rank_small's per-rank reloc attention at G = 4 and 8 under each bf16 workgroup shape
    (SR_ATTN_CFG: -1 auto, 0 = 4 waves x 2 q-blocks, 1 = 8 x 1, 2 = 2 x 2 = 128 rows), interleaved."""
    C, H, D, P, N = 1024, 16, 64, 1374, 32
    nsub = N * 305
    for G in (4, 8):
        nq = N // G
        qkv = torch.randn(nq * P + 64, 3 * C, device=DEV, dtype=torch.bfloat16)[:nq * P]
        kv = torch.randn(nsub + 64, 2 * C, device=DEV, dtype=torch.bfloat16)[:nsub]
        o = torch.empty(nq * P, C, device=DEV, dtype=torch.bfloat16)
        kb = 1.01 * max(float(qkv[:, C:2 * C].float().view(-1, H, D).norm(dim=-1).max()),
                        float(kv[:, :C].float().view(-1, H, D).norm(dim=-1).max()))
        fl = 4.0 * nq * H * P * (nsub + P) * D
        for cfg in (-1, 0, 1, 2, -1, 0, 1, 2):
            with ops.tuning(SR_ATTN_CFG=cfg):
                ms = timeit(lambda: ops.attention(qkv[:, :C], kv[:, :C], kv[:, C:], o, heads=H, head_dim=D, batch=nq,
                                                  lq=P, q_bstride=P, l0=nsub, k0_bstride=0, k1=qkv[:, C:2 * C],
                                                  v1=qkv[:, 2 * C:], l1=P, k1_bstride=P, key_norm_max=kb,
                                                  tail_readable=True))
                kern = ops.last_kernel()
            print(f"attn rank cfg G={G} reloc {nq}x({nsub}+{P}) cfg {cfg:2d} ({kern}) {ms:8.3f} ms  "
                  f"{fl / ms / 1e9:8.1f} TF/s", flush=True)


def gemm_rank():
    """The block GEMMs at the per-rank row counts of the frame-sharded C3 forward (64/G frames)."""
    for G in (1, 2, 4, 8):
        gemm(2 * 32 * 1374 // G)


def gemm(M=2 * 32 * 1374):
    for name, (N, K, epi) in {"qkv": (3072, 1024, _lib.SR_EPI_BIAS), "proj": (1024, 1024, _lib.SR_EPI_BIAS_RESID),
                              "fc1": (4096, 1024, _lib.SR_EPI_BIAS_GELU), "fc2": (1024, 4096, _lib.SR_EPI_BIAS_RESID)}.items():
        a = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
        w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) / 32
        b = torch.randn(N, device=DEV)
        g = torch.randn(N, device=DEV)
        if epi == _lib.SR_EPI_BIAS_RESID:
            out = torch.zeros(M, N, device=DEV)
        else:
            out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        ms = timeit(lambda: ops.gemm(a, w, out, epi, bias=b, gamma=g))
        fl = 2.0 * M * N * K
        print(f"gemm {name:5s} M={M} N={N} K={K} {ms:8.3f} ms  {fl / ms / 1e9:8.1f} TF/s  {fl / ms / 1e9 / PEAK:6.1%}")


def gemm_epi(M=2 * 32 * 1374):
    """fc1's shape (N = 4,096, K = 1,024) under each epilogue, interleaved: what the erf-GELU costs
    beside the plain bias epilogue, and K = 2,048 / 4,096 for the k-loop's share."""
    N = 4096
    for K in (1024, 2048, 4096):
        a = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
        w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) / 32
        b = torch.randn(N, device=DEV)
        out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        fl = 2.0 * M * N * K
        for name, epi in (("bias", _lib.SR_EPI_BIAS), ("gelu", _lib.SR_EPI_BIAS_GELU)) * 2:
            ms = timeit(lambda: ops.gemm(a, w, out, epi, bias=b))
            print(f"gemm_epi {name:4s} M={M} N={N} K={K} {ms:8.3f} ms  {fl / ms / 1e9:8.1f} TF/s", flush=True)
        del a, w


def gemm_qkv(M=2 * 32 * 1374):
    """The QKV projection at C3 rows: plain bias (DINO) against the fused qk-LayerNorm + 2-D RoPE +
    c*q epilogue (the aggregator blocks, runtime.qkv_params(prescale=True)), and the layer's grouped
    launch (queries' and anchors' QKV + the anchor-subsample K/V, sr_gemm_group)."""
    from sailrecon_amd.layers.rope import RotaryPositionEmbedding2D
    N, K, C = 3072, 1024, 1024
    a = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) / 32
    b = torch.randn(N, device=DEV)
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    rope = RotaryPositionEmbedding2D(100).tables(64, 38, DEV)
    nw = [torch.rand(64, device=DEV) + 0.5 for _ in range(4)]
    epi = dict(embed_dim=C, head_dim=64, qk_eps=1e-5, qn_w=nw[0], qn_b=nw[1] - 1, kn_w=nw[2], kn_b=nw[3] - 1,
               rope_cos=rope[0], rope_sin=rope[1], tokens_per_frame=1374, patch_start=5, grid_w=37, pos_row_base=0,
               q_scale=0.125 * 1.4426950408889634)
    fl = 2.0 * M * N * K
    ms = timeit(lambda: ops.gemm(a, w, out, _lib.SR_EPI_BIAS, bias=b))
    print(f"gemm_qkv bias              M={M} N={N} K={K} {ms:8.3f} ms  {fl / ms / 1e9:8.1f} TF/s  {fl / ms / 1e9 / PEAK:6.1%}")
    for lds in (0, 1, 0, 1):  # RoPE tables from global memory (0) or staged in LDS (1)
        with ops.tuning(SR_GEMM_ROPE_LDS=lds):
            ms = timeit(lambda: ops.gemm(a, w, out, _lib.SR_EPI_QKV, bias=b, qkv=epi))
        print(f"gemm_qkv qkv-norm-rope lds={lds} {ms:8.3f} ms  {fl / ms / 1e9:8.1f} TF/s  {fl / ms / 1e9 / PEAK:6.1%}")
    half = M // 2
    sub = torch.randint(0, half, (32 * 305,), device=DEV, dtype=torch.int32)
    kv = torch.empty(sub.numel(), 2 * C, device=DEV, dtype=torch.bfloat16)
    e_s = dict(epi, col_offset=C, pos_rowmap=sub)
    e_s.pop("pos_row_base")
    e_s.pop("q_scale")
    probs = [dict(a=a[:half], w=w, out=out[:half], bias=b, qkv=epi),
             dict(a=a[half:], w=w, out=out[half:], bias=b, qkv=dict(epi, pos_row_base=half)),
             dict(a=a[:sub.numel()], w=w[C:], out=kv, bias=b[C:], qkv=e_s)]
    flg = fl + 2.0 * sub.numel() * 2 * C * K
    for lds in (0, 1, 0, 1):
        with ops.tuning(SR_GEMM_ROPE_LDS=lds):
            ms = timeit(lambda: ops.gemm_group(probs, _lib.SR_EPI_QKV))
        print(f"gemm_qkv group (layer) lds={lds} {ms:8.3f} ms  {flg / ms / 1e9:8.1f} TF/s  {flg / ms / 1e9 / PEAK:6.1%}")


def gemm_resid():
    """SR_GEMM_RESID_LDS A/B, interleaved: the residual GEMMs (proj K=1024, fc2 K=4096) over the C3
    frame rows with the x tile staged through LDS (1) or the register epilogue (0)."""
    M, N = 2 * 32 * 1374, 1024
    x = torch.randn(M, N, device=DEV)
    b, gam = torch.randn(N, device=DEV), torch.randn(N, device=DEV) * 1e-3
    for name, K in (("proj", 1024), ("fc2 ", 4096)):
        a = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
        w = (torch.randn(N, K, device=DEV) / K ** 0.5).to(torch.bfloat16)
        fl = 2.0 * M * N * K
        for rl in (0, 1, 0, 1):
            with ops.tuning(SR_GEMM_RESID_LDS=rl):
                ms = timeit(lambda: ops.gemm(a, w, x, _lib.SR_EPI_BIAS_RESID, bias=b, gamma=gam), reps=10)
            print(f"gemm_resid {name} resid_lds={rl} {ms:.4f} ms  {fl / ms / 1e9:7.1f} TF/s", flush=True)


def gemm_k():
    """Per-tile fixed cost of the 256x256 GEMM: exactly 5 rounds of 256 tiles (M = 81,920, N = 1024)
    at K = 256 ... 4096; time = fixed + K * per-k, the intercept is the prologue / epilogue / tile
    start cost of one round."""
    M, N = 81920, 1024
    for epi, ename in ((_lib.SR_EPI_BIAS, "bias"), (_lib.SR_EPI_BIAS_RESID, "resid")):
        for K in (256, 512, 1024, 2048, 4096):
            a = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
            w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) / 32
            b = torch.randn(N, device=DEV)
            g = torch.randn(N, device=DEV)
            out = torch.zeros(M, N, device=DEV) if epi == _lib.SR_EPI_BIAS_RESID else \
                torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
            ms = timeit(lambda: ops.gemm(a, w, out, epi, bias=b, gamma=g))
            fl = 2.0 * M * N * K
            print(f"gemm_k {ename:5s} M={M} N={N} K={K:5d} {ms:8.4f} ms  {ms / 5 * 1e3:7.2f} us/round  "
                  f"{fl / ms / 1e9:8.1f} TF/s")


def gemm_f32():
    """The exact-fp32 GEMM at DPT conv shapes (im2col'd 3x3 convs, 8 frames per chunk)."""
    for name, (M, N, K) in {"rn1 3x3 256->256 @148": (8 * 148 * 148, 256, 2304),
                            "out1 3x3 256->128 @296": (8 * 296 * 296, 128, 2304),
                            "out2 3x3 128->32 @518": (8 * 518 * 518, 32, 1152)}.items():
        a = torch.randn(M, K, device=DEV)
        w = torch.randn(N, K, device=DEV) / 32
        out = torch.empty(M, N, device=DEV)
        ms = timeit(lambda: ops.gemm(a, w, out, _lib.SR_EPI_BIAS, splits=1), reps=3)
        fl = 2.0 * M * N * K
        print(f"gemm_f32 {name:24s} M={M} N={N} K={K} {ms:8.3f} ms  {fl / ms / 1e9:7.1f} TF/s  {fl / ms / 1e9 / 157.3:6.1%}")


def gemm_cam():
    """The camera trunk's fp32 weight-streaming GEMMs (camera_head.py:163-168 trunk blocks at dim 2048,
    M = 64 camera tokens at C3): time per launch and the weight-stream rate for each split-K count
    (the automatic plan marked *)."""
    M = 64
    shapes = {"qkv  ": (6144, 2048, _lib.SR_EPI_BIAS), "proj ": (2048, 2048, _lib.SR_EPI_BIAS_RESID),
              "fc1  ": (8192, 2048, _lib.SR_EPI_BIAS_GELU), "fc2  ": (2048, 8192, _lib.SR_EPI_BIAS_RESID)}
    for name, (N, K, epi) in shapes.items():
        a = torch.randn(M, K, device=DEV)
        w = torch.randn(N, K, device=DEV) / 32
        b, gam = torch.randn(N, device=DEV), torch.randn(N, device=DEV)
        out = torch.zeros(M, N, device=DEV)
        auto = ops._splitk_plan(M, N, K, epi, torch.float32)
        kt = K // 32
        for s in sorted({1, 2, 4, 8, 16, 32, 64, auto}):
            if kt % s or kt // s < 2:
                continue
            ms = timeit(lambda: ops.gemm(a, w, out, epi, bias=b, gamma=gam, splits=s), reps=20)
            print(f"gemm_cam {name} N={N} K={K} splits={s:2d}{'*' if s == auto else ' '} {ms * 1e3:8.1f} us  "
                  f"{N * K * 4 / ms / 1e9:6.2f} TB/s weights")


def torch_mm():
    """Yardstick only (not a product path): the library GEMM (torch.matmul -> hipBLASLt) at the
    block shapes, plain bf16 output, no epilogue."""
    M = 2 * 32 * 1374
    for name, (N, K) in {"qkv": (3072, 1024), "proj": (1024, 1024), "fc1": (4096, 1024), "fc2": (1024, 4096)}.items():
        a = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
        wt = (torch.randn(N, K, device=DEV, dtype=torch.bfloat16) / 32).t()
        ms = timeit(lambda: torch.matmul(a, wt))
        fl = 2.0 * M * N * K
        print(f"torch.mm {name:5s} M={M} N={N} K={K} {ms:8.3f} ms  {fl / ms / 1e9:8.1f} TF/s  {fl / ms / 1e9 / PEAK:6.1%}")


def ln():
    M, C = 2 * 32 * 1374, 1024
    x = torch.randn(M, C, device=DEV)
    w, b = torch.randn(C, device=DEV), torch.randn(C, device=DEV)
    out = torch.empty(M, C, device=DEV, dtype=torch.bfloat16)
    ms = timeit(lambda: ops.layernorm(x, w, b, 1e-5, out))
    gb = M * C * 6 / 1e9
    print(f"layernorm M={M} C={C} {ms:8.3f} ms  {gb / ms * 1e3:8.1f} GB/s")
    # the stream rate of the same bytes without the row reductions (ATen's cast copy, fp32 -> bf16):
    # the roofline the LayerNorm's 6 B per element is held against
    ms = timeit(lambda: out.copy_(x), reps=20)
    print(f"aten cast copy fp32->bf16 M={M} C={C} {ms:8.3f} ms  {gb / ms * 1e3:8.1f} GB/s")
    x2 = torch.empty_like(x)
    ms = timeit(lambda: x2.copy_(x), reps=20)
    print(f"aten copy fp32 M={M} C={C} {ms:8.3f} ms  {M * C * 8 / 1e9 / ms * 1e3:8.1f} GB/s", flush=True)
    del x2
    # x += g * y; out = LN(x) (runtime.proj_residual_ln2), y strided in the qkv slot
    ybuf = torch.randn(M, 3 * C, device=DEV).bfloat16()
    g = torch.randn(C, device=DEV) * 0.01
    ms = timeit(lambda: ops.residual_layernorm(x, ybuf[:, :C], g, w, b, 1e-5, out))
    gb = M * C * 12 / 1e9
    print(f"residual_layernorm M={M} C={C} {ms:8.3f} ms  {gb / ms * 1e3:8.1f} GB/s", flush=True)
    yc = torch.randn(M, C, device=DEV).bfloat16()  # the deferred fc2 residual: y in the o slot (ld = C)
    # SR_RLN_WIDE variants: bit 0 16-B lanes, bit 1 two rows in flight per wave, bit 2 nt x stores
    for var in (0, 1, 2, 3, 4, 6, 0, 1, 2, 3, 4, 6):
        with ops.tuning(SR_RLN_WIDE=var):
            ms = timeit(lambda: ops.residual_layernorm(x, yc, g, w, b, 1e-5, out), reps=20)
        print(f"residual_layernorm (y ld=C, variant {var}) M={M} C={C} {ms:8.3f} ms  {gb / ms * 1e3:8.1f} GB/s",
              flush=True)


def dpt():
    """DPT point + depth heads on 32 query frames @518, fp32."""
    from sailrecon_amd.heads.dpt_head import DPTHead
    from sailrecon_amd.utils.synth_weights import synth_state_dict_like
    S, H, W, C, P = 32, 518, 518, 2048, 1374
    g = torch.Generator(device=DEV).manual_seed(0)
    toks = {l: torch.randn(1, S, P, C, device=DEV, generator=g) for l in (4, 11, 17, 23)}
    images = torch.rand(1, S, 3, H, W, device=DEV, generator=g)
    for kind, kw in (("point", dict(output_dim=4, activation="inv_log")), ("depth", dict(output_dim=2, activation="exp"))):
        m = DPTHead(dim_in=C, **kw)
        m.load_state_dict(synth_state_dict_like(m))
        m = m.to(DEV)
        ms = timeit(lambda: m(toks, images=images, patch_start_idx=5), reps=2, warm=1)
        print(f"dpt {kind:5s} head S={S} @{H}  {ms:9.2f} ms  ({ms / S:.2f} ms/frame)")


def reloc():
    """Two-phase relocalisation at N=32 anchors @518 (bf16 aggregator, fp32 heads): tmp_forward
    once, then reloc() of single query views (train/demo_imc.py flow)."""
    from sailrecon_amd.models.sail_recon import SailRecon
    from sailrecon_amd.utils.synth_weights import synth_state_dict_like
    n = 32
    m = SailRecon(kv_cache=True)
    m.load_state_dict(synth_state_dict_like(m))
    m = m.to(DEV).eval()
    x = torch.rand(n, 3, 518, 518, device=DEV, generator=torch.Generator(device=DEV).manual_seed(n))
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        ms1 = timeit(lambda: m.tmp_forward(x, fix_rank=300), reps=2, warm=1)
        for flags, name in ((dict(fast_reloc=True), "pose only"), (dict(), "pose+depth"),
                            (dict(memory_save=False, ret_img=True), "all heads")):
            ms = timeit(lambda: m.reloc(x[:1], fix_rank=300, **flags), reps=5, warm=2)
            print(f"reloc 1 view vs {n} anchors @518 ({name:10s}) {ms:8.2f} ms")
    print(f"tmp_forward {n} anchors @518            {ms1:8.2f} ms")


def io():
    """Input formation: 32 views 768x1024 -> 518 (pad to square, Pillow
    BICUBIC, ToTensor), RGB and uint16 depth; kernel passes with pixels resident in HBM, then the
    whole ImagePreprocessor.process_views from PIL images (host decode arrays + H2D included),
    beside Pillow on one host core."""
    import numpy as np
    from PIL import Image
    from sailrecon_amd.utils import io as sio
    n, h, w, T = 32, 768, 1024, 518
    m, pl, pt = max(h, w), 0, (max(h, w) - h) // 2
    rng = np.random.default_rng(0)
    rgb = rng.integers(0, 256, (n, h, w, 3), dtype=np.uint8)
    dep = rng.integers(0, 65536, (n, h, w), dtype=np.uint16)
    for mode, arr, c, esz in ((sio.MODE_8BIT, rgb, 3, 1), (sio.MODE_I16, dep, 1, 2)):
        pix = sio._upload(list(arr), DEV)
        bh, kh = sio.pil_table(m, T, mode, DEV, quads=True, pad=pl, extent=w)
        bv, kv = sio.pil_table(m, T, mode, DEV, pad=pt, extent=h)
        tmp = ops.pil_tmp(n, c, h, T, pix.dtype, DEV)
        out = torch.empty(n, c, T, T, device=DEV)
        div = 255.0 if mode == sio.MODE_8BIT else 1000.0
        th_ = timeit(lambda: ops.pil_resample_h(mode, pix, bh, kh, T, tmp), reps=20)
        tv_ = timeit(lambda: ops.pil_resample_v(mode, tmp, bv, kv, div, out), reps=20)
        name = "rgb  " if mode == sio.MODE_8BIT else "depth"
        ldt = (T + 3) // 4 * 4
        bh_ = n * (h * w * c * esz + h * ldt * c * esz)
        bv_ = n * (h * ldt * c * esz + c * T * T * 4)
        ba_ = n * (h * w * c * esz + c * T * T * 4)
        print(f"io {name} h pass {th_ * 1e3:8.1f} us  {bh_ / th_ / 1e6:7.1f} GB/s   "
              f"v pass {tv_ * 1e3:8.1f} us  {bv_ / tv_ / 1e6:7.1f} GB/s   ({(th_ + tv_) / n * 1e3:.1f} us/view; "
              f"in+out {ba_ / n / 1e6:.2f} MB/view -> {ba_ / (th_ + tv_) / 1e6:.0f} GB/s)")
    pre = sio.ImagePreprocessor(T, device=DEV)
    ims = [Image.fromarray(a) for a in rgb]
    dims = [Image.fromarray(a) for a in dep]
    ms = timeit(lambda: pre.process_views(ims), reps=3, warm=1)
    msd = timeit(lambda: pre.process_views(dims, is_depth=True), reps=3, warm=1)
    print(f"io process_views from PIL (incl. host arrays + H2D): rgb {ms / n:.3f} ms/view  depth {msd / n:.3f} ms/view")
    t0 = time.perf_counter()
    for im in ims[:8]:
        sq = Image.new("RGB", (m, m))
        sq.paste(im, (pl, pt))
        np.asarray(sq.resize((T, T), Image.Resampling.BICUBIC), dtype=np.float32) / 255
    t1 = time.perf_counter()
    for im in dims[:4]:
        sq = Image.new(im.mode, (m, m))
        sq.paste(im, (pl, pt))
        np.asarray(sq.resize((T, T), Image.Resampling.BICUBIC)).astype(np.float32) / 1000
    t2 = time.perf_counter()
    print(f"io Pillow on 1 host core: rgb {(t1 - t0) / 8 * 1e3:.2f} ms/view  depth {(t2 - t1) / 4 * 1e3:.2f} ms/view")


def attn_fp8():
    """Global attention with q.k^T in block-scaled fp8 (BASELINE C5) vs the bf16 kernel, at the
    C3 (L = 43,968) and C5 (L = 175,872) global lengths; the fp8 time includes both quantisations."""
    C, H, D, P = 1024, 16, 64, 1374
    for n in (32, 128):
        L = n * P
        qkv = torch.randn(L, 3 * C, device=DEV, dtype=torch.bfloat16)
        o = torch.empty(L, C, device=DEV, dtype=torch.bfloat16)
        ws = ops.Fp8Workspace()
        fl = 4.0 * H * L * L * D
        kb = float(qkv[:, C:2 * C].float().view(-1, H, D).norm(dim=-1).max())  # the static key bound's role
        for name, f in (("bf16", lambda: ops.attention(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], o, heads=H, head_dim=D,
                                                        batch=1, lq=L, q_bstride=0, l0=L, k0_bstride=0,
                                                        key_norm_max=kb)),
                        ("fp8 qk", lambda: ops.attention_qk8(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], o, heads=H,
                                                           batch=1, lq=L, q_bstride=0, l0=L, k0_bstride=0, ws=ws,
                                                           key_norm_max=kb)),
                        ("fp8 qkv", lambda: ops.attention_qk8(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], o, heads=H,
                                                            batch=1, lq=L, q_bstride=0, l0=L, k0_bstride=0, ws=ws,
                                                            fp8_v=True))):
            ms = timeit(f, reps=3 if n == 128 else 5, warm=1)
            print(f"attn global L={L:6d} {name:7s} {ms:9.3f} ms  {fl / ms / 1e9:8.1f} TF/s", flush=True)


def attn_bwd():
    """Attention backward at the training shapes (C4: 16 anchors -> global L = 21984; frames; the
    reloc block: 16 query frames against SR_BWD_RELOC_ANCHORS shared anchor keys + their own frame)."""
    C, H, D, P = 1024, 16, 64, 1374
    na = int(os.environ.get("SR_BWD_RELOC_ANCHORS", "9984"))
    shapes = [("global L=21984", 16 * P, 1, 16 * P, 0), ("frame 32x1374", 32 * P, 32, P, 0)]
    if os.environ.get("SR_BWD_RELOC", "1") != "0":
        shapes.append((f"reloc 16x{P}+{na}", 16 * P, 16, P, na))
    for name, rows, batch, lq, anchors in shapes:
        qkv = torch.randn(rows, 3 * C, device=DEV, dtype=torch.bfloat16)
        o = torch.empty(rows, C, device=DEV, dtype=torch.bfloat16)
        lse = torch.empty(batch, H, lq, device=DEV)
        kb = 0 if batch == 1 else lq
        if anchors:  # segment 0: anchor keys shared by every item; segment 1: the item's own frame
            akv = torch.randn(anchors, 2 * C, device=DEV, dtype=torch.bfloat16)
            seg = dict(k0=akv[:, :C], v0=akv[:, C:], l0=anchors, k0_bstride=0, l1=lq, k1_bstride=lq)
            dka = torch.empty(anchors, 2 * C, device=DEV)
        else:
            seg = dict(k0=qkv[:, C:2 * C], v0=qkv[:, 2 * C:], l0=lq, k0_bstride=kb)
        fwd_kw = dict(seg)
        k0, v0 = fwd_kw.pop("k0"), fwd_kw.pop("v0")
        if anchors:
            fwd_kw.update(k1=qkv[:, C:2 * C], v1=qkv[:, 2 * C:])
        ops.attention(qkv[:, :C], k0, v0, o, heads=H, head_dim=D, batch=batch, lq=lq, q_bstride=lq, lse=lse,
                      **fwd_kw)
        g = torch.randn(rows, C, device=DEV, dtype=torch.bfloat16)
        d = torch.empty(rows, 3 * C, device=DEV)
        delta = torch.empty(batch * H * lq, device=DEV)

        def f():
            if anchors:
                ops.attention_bwd(qkv[:, :C], k0, v0, o, lse, g, d[:, :C], dka[:, :C], dka[:, C:], delta, heads=H,
                                  batch=batch, lq=lq, q_bstride=lq, dk1=d[:, C:2 * C], dv1=d[:, 2 * C:], **fwd_kw)
            else:
                ops.attention_bwd(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], o, lse, g, d[:, :C], d[:, C:2 * C],
                                  d[:, 2 * C:], delta, heads=H, batch=batch, lq=lq, q_bstride=lq, l0=lq, k0_bstride=kb)
        fl = 10.0 * batch * H * lq * (lq + anchors) * D  # S, dP, dV, dK, dQ (flash-attention backward convention)
        # compiled sweeps (kb1), the asm sweeps (pipe2), + the concatenated-items dK/dV sweep (cat)
        arms = [("kb1", dict(SR_ATTN_BWD_PIPE=0, SR_ATTN_BWD_DQ_PIPE=0, SR_ATTN_BWD_CAT=0)),
                ("pipe2", dict(SR_ATTN_BWD_PIPE=1, SR_ATTN_BWD_DQ_PIPE=1, SR_ATTN_BWD_CAT=0)),
                ("cat", dict(SR_ATTN_BWD_PIPE=1, SR_ATTN_BWD_DQ_PIPE=1, SR_ATTN_BWD_CAT=1))]
        if os.environ.get("SR_BWD_AB") == "pipe":  # the asm sweeps only (A/B of library builds)
            arms = arms[1:2]
        for arm, sw in arms * 2:
            with ops.tuning(**sw):
                ms = timeit(f, reps=3 if batch == 1 else 5, warm=1)
            print(f"attn_bwd {name:16s} {arm:5s} {ms:8.3f} ms  {fl / ms / 1e9:8.1f} TF/s  {fl / ms / 1e9 / PEAK:6.1%}",
                  flush=True)


def qk_bwd():
    """sr_qk_bwd at the C4 frame block's shape (43,968 rows, q|k|v 3,072 columns, qk-norm + RoPE):
    plain, plain + the bf16 column sum of its output (the qkv bias grad, as before round 6), and
    with the column sum from the same pass (bias_grad)."""
    from sailrecon_amd.layers.rope import RotaryPositionEmbedding2D
    R, C, D = 32 * 1374, 1024, 64
    g = torch.Generator(device=DEV).manual_seed(3)
    raw = torch.randn(R, 3 * C, device=DEV, generator=g).bfloat16()
    dsrc = torch.randn(R, 3 * C, device=DEV, generator=g)
    out = torch.empty(R, 3 * C, device=DEV, dtype=torch.bfloat16)
    rope = RotaryPositionEmbedding2D(100).tables(D, 37, DEV)
    epi = dict(embed_dim=C, head_dim=D, qk_eps=1e-6, qn_w=torch.randn(D, device=DEV), qn_b=torch.randn(D, device=DEV),
               kn_w=torch.randn(D, device=DEV), kn_b=torch.randn(D, device=DEV), rope_cos=rope[0], rope_sin=rope[1],
               tokens_per_frame=1374, patch_start=5, grid_w=37, pos_row_base=0)
    grads = torch.zeros(4, 64, device=DEV)
    bg = torch.zeros(3 * C, device=DEV)

    def plain():
        ops.qk_bwd(raw, dsrc, out, epi, grads=grads)

    def plain_cs():
        ops.qk_bwd(raw, dsrc, out, epi, grads=grads)
        ops.colsum(out, bg, accumulate=True)

    def fused():
        ops.qk_bwd(raw, dsrc, out, epi, grads=grads, bias_grad=bg)
    for i in range(2):
        tp, tc, tf = timeit(plain, reps=20), timeit(plain_cs, reps=20), timeit(fused, reps=20)
        print(f"qk_bwd C4 frame rows: plain {tp * 1e3:.1f} us, plain + colsum {tc * 1e3:.1f} us, "
              f"fused colsum {tf * 1e3:.1f} us", flush=True)


def train():
    """BASELINE config 4 (train_imc.py step, 16-view batches): full-size SailRecon aggregator +
    camera head (DPT heads off: no loss reaches them), seeded synthetic weights, a synthetic
    16-view IMC-shaped batch (15 chained pairs x 1024 correspondences, per-frame CDF nodes), bf16
    aggregator / fp32 heads, fwd + loss + bwd + Adam per step.  SR_TRAIN_QK_GAIN=g scales every
    q_norm / k_norm weight by g first (trained-like gains)."""
    from sailrecon_amd.models.sail_recon import SailRecon
    from sailrecon_amd.train.data import synthetic_batch
    from sailrecon_amd.train.loss import CDFLossIndexPytorch
    from sailrecon_amd.train.step import Trainer, prepare_model_input
    from sailrecon_amd.utils.synth_weights import synth_state_dict_like
    n = int(os.environ.get("SR_TRAIN_VIEWS", "16"))
    steps = int(os.environ.get("SR_TRAIN_STEPS", "3"))
    t0 = time.perf_counter()
    m = SailRecon(enable_point=False, enable_depth=False)
    m.load_state_dict(synth_state_dict_like(m), strict=False)
    gain = float(os.environ.get("SR_TRAIN_QK_GAIN", "1"))
    if gain != 1.0:  # trained-like q_norm / k_norm weights (bench.py --qk-gain)
        with torch.no_grad():
            for mod in m.modules():
                for nm in ("q_norm", "k_norm"):
                    ln = getattr(mod, nm, None)
                    if ln is not None and getattr(ln, "weight", None) is not None:
                        ln.weight.mul_(gain)
    m = m.to(DEV)
    print(f"train: model built in {time.perf_counter() - t0:.1f} s (qk-norm gain {gain:g})", flush=True)
    b = synthetic_batch(n, n_points=1024, size=518, seed=0)
    cdf = CDFLossIndexPytorch(0.0, 15.0, 250, b["src_idx"], b["dst_idx"], gradient_smooth=0.05, num_nodes=n)
    tr = Trainer(m, max_lr=2e-4, warmup_steps=2000, max_steps=100_000, cdf=cdf)
    imgs, na, nq = prepare_model_input(b["rgb_processed"].to(DEV))
    ops.TIMER = ops.KernelTimer()
    out = tr.step(imgs, na, nq, b)  # warmup (allocates tapes / packs)
    torch.cuda.synchronize()
    print(f"train: warmup step loss {out['loss']:.5f}  peak HBM {torch.cuda.max_memory_allocated() / 2**30:.1f} GiB",
          flush=True)
    # the step time without instrumentation (the per-op HIP events of ops.KernelTimer cost host time,
    # and the backward's short launches run where the host is only just ahead), then the same steps
    # again under the kernel timer for the per-class breakdown
    ops.TIMER = None
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(steps):
        out = tr.step(imgs, na, nq, b)
    ev[1].record()
    torch.cuda.synchronize()
    ms = ev[0].elapsed_time(ev[1]) / steps
    ops.TIMER = ops.KernelTimer()
    ev[0].record()
    for _ in range(steps):
        tr.step(imgs, na, nq, b)
    ev[1].record()
    torch.cuda.synchronize()
    ms_timed = ev[0].elapsed_time(ev[1]) / steps
    summ = ops.TIMER.summary()
    ops.TIMER = None
    tot = 0.0
    for tag, r in sorted(summ.items(), key=lambda kv: -kv[1]["total_ms"]):
        tot += r["total_ms"] / steps
        print(f"  {tag:22s} {r['total_ms'] / steps:9.2f} ms/step  {r['launches'] // steps:5d} launches  "
              f"{r['tflops']:7.1f} TF/s")
    print(f"train: {n} views ({2 * n} frames @518) {ms:.1f} ms/step = {n / ms * 1e3:.2f} views/s "
          f"({1e3 / ms:.3f} steps/s); under the kernel timer {ms_timed:.1f} ms/step, timed kernels {tot:.1f} ms; "
          f"loss {out['loss']:.5f}", flush=True)
    # the box's calibration GEMM (bench.py box_calibration), so that steps from different boxes compare
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
    from bench import box_calibration
    cal = box_calibration(torch.device(DEV))
    print(f"train: box calibration {cal['tflops']} TF/s ({cal['kernel']}, {cal['shape']})", flush=True)


if __name__ == "__main__":
    which = sys.argv[1:] or ["attn", "gemm", "ln"]
    for w in which:
        globals()[w]()
