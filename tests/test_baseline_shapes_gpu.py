"""The attention kernels at the BASELINE workloads' exact launch shapes.

Each launch runs at its production size; ~256 sampled query rows per head are checked against
fp64 softmax attention over ALL of the keys those rows attend to (the full sweep, every ragged
tile and every late-tile rescale included).  Inputs: q and k per-head layer-normalised like the
aggregator's qk-norm (attention.py:78) with a spread of gains, V normal; a few "spike" keys late
in the sequence score far above the rest, so the online softmax must move its running max (or
use its overflow-safe bound) deep into the sweep (cdna_hip_programming.md §5.4 rule 26).

Shapes (P = 1374 tokens per frame at 518 px, P' = 305 subsample rows per anchor):
  global   L_g = N·P:        C2 10,992   C3 43,968   C5 175,872   (one item, 16 heads)
  reloc    Nq frames × P queries against [N·P' shared subsample ; own frame]:
           C2 8 × 1374 vs 2,440 + 1374      C3 32 × 1374 vs 9,760 + 1374
  frame    S = 2N frames × P, keys = own frame: C3 64 × 1374
Tolerances: bf16 operands in, fp64 reference on the SAME bf16 operands: 1e-2 rel-L2 (P is rounded
to bf16 for the P·V product).  fp8 modes against fp64 on the dequantised q8/k8 (and V8): 1e-2 /
3e-2 as in test_fp8_gpu.py; against the exact attention (the fp8 rounding itself, parity
unpinned: the reference has no fp8 path) 0.15, the measured values printed.
"""

import math

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"
H, D = 16, 64
C = H * D
P, PP = 1374, 305


def _rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


@pytest.fixture(scope="module")
def ops():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from sailrecon_amd import ops as _ops
    return _ops


def _qk_normed(rows, gen, gain_lo=0.5, gain_hi=2.0):
    """[rows, C] bf16: per-head LayerNorm'd gaussian times a per-head gain (qk-norm-like)."""
    x = torch.randn(rows, H, D, device=DEV, generator=gen)
    x = (x - x.mean(-1, keepdim=True)) / x.std(-1, keepdim=True, unbiased=False)
    gain = torch.linspace(gain_lo, gain_hi, H, device=DEV)[None, :, None]
    return (x * gain).reshape(rows, C).bfloat16()


def _make(rows, seed, spikes=()):
    """q carries half of a shared per-head direction u (|u| = 8); a spike key 3u then scores
    about 12 (natural log) above the typical key for EVERY query row."""
    g = torch.Generator(device=DEV).manual_seed(seed)
    u = torch.randn(H, D, device=DEV, generator=g)
    u = (u * (D ** 0.5) / u.norm(dim=-1, keepdim=True)).reshape(C)
    q = (_qk_normed(rows, g).float() + 0.5 * u).bfloat16()
    k = _qk_normed(rows, g)
    v = torch.randn(rows, C, device=DEV, generator=g).bfloat16()
    for r in spikes:
        k[r] = (3.0 * u).bfloat16()
    return q, k, v


def _sample_rows(lq, n, seed):
    g = torch.Generator().manual_seed(seed)
    rows = torch.randperm(lq, generator=g)[:n]
    return torch.sort(torch.cat([rows, torch.tensor([0, lq - 1])]).unique()).values


def _ref_rows(qs, ks, vs, scale):
    """fp64 attention of qs [n, C] over keys ks/vs [L, C], per head -> [n, C]."""
    out = torch.empty(qs.shape[0], C, dtype=torch.float64, device=DEV)
    for h in range(H):
        c = slice(h * D, (h + 1) * D)
        s = (qs[:, c].double() @ ks[:, c].double().T) * scale
        out[:, c] = torch.softmax(s, -1) @ vs[:, c].double()
    return out


@pytest.mark.parametrize("L", [10_992, 43_968, 87_936, 175_872], ids=["C2", "C3", "N64", "C5"])
def test_global_attention_production(ops, L):
    q, k, v = _make(L, 7, spikes=(L - 37, L // 2 + 5))
    o = torch.empty(L, C, device=DEV, dtype=torch.bfloat16)
    ops.attention(q, k, v, o, heads=H, head_dim=D, batch=1, lq=L, q_bstride=0, l0=L, k0_bstride=0)
    rows = _sample_rows(L, 256, L).to(DEV)
    ref = _ref_rows(q[rows], k, v, D ** -0.5)
    assert _rel(o[rows].float(), ref) < 1e-2


def _kbound(k, heads=H):
    return 1.01 * float(k.float().view(k.shape[0], heads, -1).norm(dim=-1).max())


@pytest.mark.parametrize("case", ["C3", "padded"])
def test_attention_pair(ops, case):
    """sr_attention_pair (ops.attention_pair): the global block's attention and the split reloc's
    subsample pass in ONE launch of the hand-scheduled sweep -- bit-identical to the two launches
    apart (outputs and the second problem's LSE), and equal to fp64 on sampled rows.  'padded': 3
    heads, so the first problem's 63 workgroups are padded to 64 (the padding workgroups exit)."""
    if case == "C3":
        heads, La, rows, nk = H, 32 * P, 32 * P, 32 * PP // 64 * 64
        qg, kg, vg = _make(La, 11, spikes=(La - 5, 77))
        qr, _, _ = _make(rows, 12)
        _, ks, vs = _make(nk, 13, spikes=(nk - 1,))
    else:
        heads, La, rows, nk = 3, 21 * 256 - 128, 9 * 256 + 7, 40 * 64  # 21 q-tiles x 3 heads = 63 workgroups
        g = torch.Generator(device=DEV).manual_seed(5)
        mk = lambda n: (torch.randn(n, heads * D, device=DEV, generator=g) * 0.5).bfloat16()  # noqa: E731
        qg, kg, vg, qr, ks, vs = mk(La), mk(La), mk(La), mk(rows), mk(nk), mk(nk)
    cols = heads * D
    kbg, kbr = _kbound(kg, heads), _kbound(ks, heads)
    og, orr = (torch.empty(n, cols, device=DEV, dtype=torch.bfloat16) for n in (La, rows))
    lse = torch.empty(heads, rows, device=DEV)
    ops.attention_pair(dict(q=qg, k0=kg, v0=vg, o=og, lq=La, l0=La, key_norm_max=kbg),
                       dict(q=qr, k0=ks, v0=vs, o=orr, lq=rows, l0=nk, key_norm_max=kbr, lse=lse.view(-1)),
                       heads=heads, head_dim=D)
    if case == "C3":  # apart, both launches take the same hand-scheduled sweep (2,752 workgroups each)
        og1, or1 = torch.empty_like(og), torch.empty_like(orr)
        lse1 = torch.empty_like(lse)
        ops.attention(qg, kg, vg, og1, heads=heads, head_dim=D, batch=1, lq=La, q_bstride=0, l0=La, k0_bstride=0,
                      key_norm_max=kbg)
        ops.attention(qr, ks, vs, or1, heads=heads, head_dim=D, batch=1, lq=rows, q_bstride=0, l0=nk,
                      k0_bstride=0, key_norm_max=kbr, lse=lse1.view(-1))
        torch.cuda.synchronize()
        assert torch.equal(og, og1) and torch.equal(orr, or1) and torch.equal(lse, lse1)
    scale = D ** -0.5
    for q_, k_, v_, o_, n in ((qg, kg, vg, og, La), (qr, ks, vs, orr, rows)):
        rws = _sample_rows(n, 64, n).to(DEV)
        ref = torch.empty(rws.numel(), cols, dtype=torch.float64, device=DEV)
        for h in range(heads):
            c = slice(h * D, (h + 1) * D)
            sc = (q_[rws][:, c].double() @ k_[:, c].double().T) * scale
            ref[:, c] = torch.softmax(sc, -1) @ v_[:, c].double()
            if o_ is orr:  # the LSE (log2 domain) of the second problem; the kernel sums the bf16-rounded
                # P that P.V uses (matrix-pipe row sums), 2^-9 relative per term: 1.5e-2 measured here
                l2 = torch.logsumexp(sc, -1) / math.log(2.0)
                assert float((lse[h, rws].double() - l2).abs().max()) < 3e-2
        assert _rel(o_[rws].float(), ref) < 1e-2


@pytest.mark.parametrize("loose", [1.0, 3.0])
@pytest.mark.parametrize("case", ["global-C3", "frame-C3"])
def test_attention_static_key_bound(ops, case, loose):
    """sr_attn_desc.key_norm_max (runtime.key_norm_bound for qk-norm blocks): a static bound of
    |k| replaces the key scan of the fixed-offset sweep.  Tight (the true max) and 3x loose bounds
    give the scan's result (same kernel, same arithmetic up to the offset) and match fp64."""
    frames = 1 if case.startswith("global") else 64
    L = 32 * P if frames == 1 else P
    q, k, v = _make(frames * L, 13, spikes=(frames * L - 37, L // 2 + 5))
    kmax = float(k.float().view(-1, H, D).norm(dim=-1).max()) * 1.01
    outs = []
    for kb in (0.0, kmax * loose):
        o = torch.empty(frames * L, C, device=DEV, dtype=torch.bfloat16)
        ops.attention(q, k, v, o, heads=H, head_dim=D, batch=frames, lq=L, q_bstride=L, l0=L, k0_bstride=L,
                      key_norm_max=kb)
        outs.append(o)
    torch.cuda.synchronize()
    assert _rel(outs[1].float(), outs[0].float()) < 5e-3
    rows = _sample_rows(L, 128, 7).to(DEV)
    f = frames - 1  # the last item (spike key 37 rows from its end)
    ref = _ref_rows(q[f * L + rows], k[f * L:(f + 1) * L], v[f * L:(f + 1) * L], D ** -0.5)
    assert _rel(outs[1][f * L + rows].float(), ref) < 1e-2


@pytest.mark.parametrize("G,r", [(2, 0), (2, 1), (3, 1)], ids=["C3-2rk-r0", "C3-2rk-r1", "C3-3rk-mid"])
def test_global_attention_sharded_passes(ops, G, r):
    """The frame-sharded global block at C3 (32 anchors): rank r's query rows attend to its own
    anchors (local pass), then to every other rank's (remote pass: one key segment at the ends,
    two — before and after the local slice — on a middle rank; 32 over 3 ranks is the uneven
    11 / 11 / 10 split), merged by sr_attn_merge.  Checked against fp64 attention over ALL keys
    and against the kernel's single pass over all keys, LSE included."""
    from sailrecon_amd.models.aggregator import shard_range
    L = 32 * P
    q, k, v = _make(L, 11, spikes=(L - 37, 3 * P + 5))
    a0, na = shard_range(32, G, r)
    off, lq = a0 * P, na * P
    qs = q[off:off + lq]
    lse_a = torch.empty(H, lq, device=DEV)
    lse_b = torch.empty(H, lq, device=DEV)
    o = torch.empty(lq, C, device=DEV, dtype=torch.bfloat16)
    o_b = torch.empty_like(o)
    ops.attention(qs, k[off:off + lq], v[off:off + lq], o, heads=H, head_dim=D, batch=1, lq=lq, q_bstride=0,
                  l0=lq, k0_bstride=0, lse=lse_a)
    segs = [(s, n) for s, n in ((0, off), (off + lq, L - off - lq)) if n > 0]
    (s0, n0), (s1, n1) = segs[0], (segs[1] if len(segs) > 1 else (0, 0))
    ops.attention(qs, k[s0:s0 + n0], v[s0:s0 + n0], o_b, heads=H, head_dim=D, batch=1, lq=lq, q_bstride=0, l0=n0,
                  k0_bstride=0, k1=k[s1:s1 + n1] if n1 else None, v1=v[s1:s1 + n1] if n1 else None, l1=n1,
                  k1_bstride=0, lse=lse_b)
    lse_m = torch.empty(H, lq, device=DEV)
    ops.attn_merge(o, lse_a, o_b, lse_b, o, heads=H, head_dim=D, lse_out=lse_m)  # in place on o
    one = torch.empty_like(o)
    lse_1 = torch.empty(H, lq, device=DEV)
    ops.attention(qs, k, v, one, heads=H, head_dim=D, batch=1, lq=lq, q_bstride=0, l0=L, k0_bstride=0, lse=lse_1)
    torch.cuda.synchronize()
    rows = _sample_rows(lq, 256, lq + G).to(DEV)
    ref = _ref_rows(qs[rows], k, v, D ** -0.5)
    assert _rel(o[rows].float(), ref) < 1e-2
    assert _rel(o.float(), one.float()) < 1e-2
    # row sums accumulate the bf16-rounded P of the P.V product: ~2^-9 per dominant term
    assert float((lse_m - lse_1).abs().max()) < 1e-2


@pytest.mark.parametrize("alias", [False, True])
def test_attn_merge_fp32_exact(ops, alias):
    """fp32 kernel passes over a 3-way key split, merged pairwise (lse_out chaining): equal to the
    one-pass fp32 kernel to float rounding; the fp32 kernel's LSE equals torch.logsumexp."""
    g = torch.Generator(device=DEV).manual_seed(3)
    lq, L, h, d = 300, 900, 6, 64
    q, k, v = (torch.randn(n, h * d, device=DEV, generator=g) for n in (lq, L, L))
    cuts = [(0, 250), (250, 610), (610, 900)]
    outs, lses = [], []
    for a, b in cuts:
        o = torch.empty(lq, h * d, device=DEV)
        lse = torch.empty(h, lq, device=DEV)
        ops.attention(q, k[a:b], v[a:b], o, heads=h, head_dim=d, batch=1, lq=lq, q_bstride=0, l0=b - a,
                      k0_bstride=0, lse=lse)
        outs.append(o)
        lses.append(lse)
    o, lse = outs[0], lses[0]
    for ob, lb in zip(outs[1:], lses[1:]):
        dst = o if alias else torch.empty_like(o)
        lse_dst = lse if alias else torch.empty_like(lse)
        ops.attn_merge(o, lse, ob, lb, dst, heads=h, head_dim=d, lse_out=lse_dst)
        o, lse = dst, lse_dst
    one = torch.empty(lq, h * d, device=DEV)
    lse1 = torch.empty(h, lq, device=DEV)
    ops.attention(q, k, v, one, heads=h, head_dim=d, batch=1, lq=lq, q_bstride=0, l0=L, k0_bstride=0, lse=lse1)
    s = torch.einsum("qhd,khd->hqk", q.view(lq, h, d).double(), k.view(L, h, d).double()) * d ** -0.5
    ref_lse = torch.logsumexp(s, -1) / math.log(2.0)
    torch.cuda.synchronize()
    assert _rel(o, one) < 1e-5
    assert float((lse1.double() - ref_lse).abs().max()) < 1e-4
    assert float((lse.double() - ref_lse).abs().max()) < 1e-4


LOG2E = 1.0 / math.log(2.0)
LN2 = math.log(2.0)  # (c q).k * ln 2 = scale q.k: the natural-log scores of a q_scaled operand


def _prescale(q):
    """What the QKV GEMM hands the attention (runtime.q_prescale, sr_attn_desc.q_scaled): c*q with
    c = scale*log2(e), rounded to bf16 ONCE from the fp32 value (here q's own values)."""
    return (q.float() * (D ** -0.5 * LOG2E)).bfloat16()


@pytest.mark.parametrize("G", [3, 8], ids=["C3-3rk", "C3-8rk"])
def test_global_attention_key_split(ops, G):
    """Key-split attention (ops.key_split_parts): one rank's query slice of the frame-sharded C3
    global block against all 43,968 keys runs as S key chunks whose bf16 partials and LSEs merge
    with sr_attn_merge_n.  Equal to the unsplit kernel (output and LSE) and to fp64 attention.
    q arrives as the production path hands it over: c*q rounded once (q_scaled), so the fp64
    reference reads the same operand, (c q).k ln 2 = scale q.k."""
    L = 32 * P
    lq = (32 // G) * P
    q, k, v = _make(L, 17, spikes=(L - 37, 5 * P + 3))
    qs = _prescale(q[L - lq:])
    parts = ops.key_split_parts(dtype=torch.bfloat16, batch=1, lq=lq, heads=H, l0=L, l1=0, mask_mode=0)
    assert parts > 1
    outs, lses = [], []
    saved = ops._KSPLIT_ENV
    try:
        for split in ("0", None):
            ops._KSPLIT_ENV = split
            o = torch.empty(lq, C, device=DEV, dtype=torch.bfloat16)
            lse = torch.empty(H, lq, device=DEV)
            ops.attention(qs, k, v, o, heads=H, head_dim=D, batch=1, lq=lq, q_bstride=0, l0=L, k0_bstride=0,
                          lse=lse, key_norm_max=float(k.float().view(-1, H, D).norm(dim=-1).max()) * 1.01,
                          q_scaled=True)
            outs.append(o)
            lses.append(lse)
    finally:
        ops._KSPLIT_ENV = saved
    torch.cuda.synchronize()
    assert _rel(outs[1].float(), outs[0].float()) < 1e-2
    rows = _sample_rows(lq, 256, G).to(DEV)
    ref = _ref_rows(qs[rows], k, v, LN2)
    # fp64 log2-domain LSE of the sampled rows over the same operands.  Round 4 re-rounded c*q inside
    # the kernel (c * bf16(q) to bf16 again), which put 5.0e-2 / 3.8e-2 of score error on the spike
    # rows and needed a 6e-2 bound; with q rounded once what is left is the row sums over the
    # bf16-rounded P of the P.V product (2^-9 per dominant term)
    s_ref = torch.einsum("qhd,khd->hqk", qs[rows].view(-1, H, D).double(), k.view(-1, H, D).double()) * LN2
    ref_lse = torch.logsumexp(s_ref, -1) / math.log(2.0)
    e_split = float((lses[1][:, rows].double() - ref_lse).abs().max())
    e_one = float((lses[0][:, rows].double() - ref_lse).abs().max())
    e_pair = float((lses[1] - lses[0]).abs().max())
    print(f"key split S={parts}: rel {_rel(outs[1][rows].float(), ref):.2e} (unsplit "
          f"{_rel(outs[0][rows].float(), ref):.2e}); LSE vs fp64 {e_split:.2e} (unsplit {e_one:.2e}), "
          f"split vs unsplit {e_pair:.2e}")
    assert _rel(outs[1][rows].float(), ref) < 1e-2
    assert e_split < 2e-2 and e_one < 2e-2 and e_pair < 2e-2


@pytest.mark.parametrize("L", [43_968, 175_872], ids=["C3", "C5"])
def test_global_attention_q_scaled(ops, L):
    """sr_attn_desc.q_scaled (the production convention since round 5): q holds c*q rounded once,
    the kernel uses it as is.  Against fp64 over the same operand at C3 / C5, the pair launch with
    q_scaled bit-identical to its two launches apart, and the plain-q launch (the kernel forms
    bf16(c * bf16(q)), a second rounding) within its own larger error."""
    q, k, v = _make(L, 23, spikes=(L - 37, L // 2 + 5))
    qs = _prescale(q)
    kb = _kbound(k)
    o = torch.empty(L, C, device=DEV, dtype=torch.bfloat16)
    o_plain = torch.empty_like(o)
    ops.attention(qs, k, v, o, heads=H, head_dim=D, batch=1, lq=L, q_bstride=0, l0=L, k0_bstride=0, key_norm_max=kb,
                  q_scaled=True)
    ops.attention(q, k, v, o_plain, heads=H, head_dim=D, batch=1, lq=L, q_bstride=0, l0=L, k0_bstride=0,
                  key_norm_max=kb)
    rows = _sample_rows(L, 256, L + 1).to(DEV)
    e_scaled = _rel(o[rows].float(), _ref_rows(qs[rows], k, v, LN2))
    e_plain = _rel(o_plain[rows].float(), _ref_rows(q[rows], k, v, D ** -0.5))
    print(f"q_scaled L={L}: rel vs fp64 {e_scaled:.2e} (plain q, re-rounded in the kernel: {e_plain:.2e})")
    assert e_scaled < 1e-2 and e_plain < 1e-2
    if L == 43_968:
        o1, o2 = torch.empty_like(o), torch.empty_like(o)
        ops.attention_pair(dict(q=qs, k0=k, v0=v, o=o1, lq=L, l0=L, key_norm_max=kb, q_scaled=True),
                           dict(q=q, k0=k, v0=v, o=o2, lq=L, l0=L, key_norm_max=kb), heads=H, head_dim=D)
        torch.cuda.synchronize()
        assert torch.equal(o1, o) and torch.equal(o2, o_plain)


def test_attn_merge_n_seg_rows_fp32(ops):
    """sr_attn_merge_n with mixed LSE layouts: two key chunks of a shared segment over 3 items' query
    rows as one set ([heads][rows]) plus the items' own segments as a batch launch
    ([items][heads][lq]) equal the two-segment fp32 kernel (global_reloc's shape)."""
    g = torch.Generator(device=DEV).manual_seed(6)
    nb, lq, ls, lo, h, d = 3, 150, 400, 120, 4, 64
    q = torch.randn(nb * lq, h * d, device=DEV, generator=g)
    ks, vs = (torch.randn(ls, h * d, device=DEV, generator=g) for _ in range(2))
    ko, vo = (torch.randn(nb * lo, h * d, device=DEV, generator=g) for _ in range(2))
    rows = nb * lq
    o_parts = torch.empty(3 * rows, h * d, device=DEV)
    lse_parts = torch.empty(3, h, rows, device=DEV)
    for p in range(2):
        ops.attention(q, ks[p * 200:(p + 1) * 200], vs[p * 200:(p + 1) * 200], o_parts[p * rows:(p + 1) * rows],
                      heads=h, head_dim=d, batch=1, lq=rows, q_bstride=0, l0=200, k0_bstride=0, lse=lse_parts[p])
    ops.attention(q, ko, vo, o_parts[2 * rows:], heads=h, head_dim=d, batch=nb, lq=lq, q_bstride=lq, l0=lo,
                  k0_bstride=lo, lse=lse_parts[2])
    o = torch.empty(rows, h * d, device=DEV)
    ops.attn_merge_n(o_parts, lse_parts, o, parts=3, rows=rows, heads=h, head_dim=d, seg_rows=[rows, rows, lq])
    one = torch.empty_like(o)
    ops.attention(q, ks, vs, one, heads=h, head_dim=d, batch=nb, lq=lq, q_bstride=lq, l0=ls, k0_bstride=0, k1=ko,
                  v1=vo, l1=lo, k1_bstride=lo)
    torch.cuda.synchronize()
    assert _rel(o, one) < 1e-5


def test_attn_merge_n_fp32_exact(ops):
    """sr_attn_merge_n over 4 equal fp32 key chunks (a key-split layout: partial p at rows p*lq,
    LSE [parts, heads, lq]) equals the one-pass fp32 kernel to float rounding, LSE included."""
    g = torch.Generator(device=DEV).manual_seed(5)
    lq, L, h, d, S = 200, 800, 4, 64, 4
    q, k, v = (torch.randn(n, h * d, device=DEV, generator=g) for n in (lq, L, L))
    o_parts = torch.empty(S * lq, h * d, device=DEV)
    lse_parts = torch.empty(S, h, lq, device=DEV)
    ch = L // S
    for p in range(S):
        ops.attention(q, k[p * ch:(p + 1) * ch], v[p * ch:(p + 1) * ch], o_parts[p * lq:(p + 1) * lq], heads=h,
                      head_dim=d, batch=1, lq=lq, q_bstride=0, l0=ch, k0_bstride=0, lse=lse_parts[p])
    o = torch.empty(lq, h * d, device=DEV)
    lse = torch.empty(h, lq, device=DEV)
    ops.attn_merge_n(o_parts, lse_parts, o, parts=S, rows=lq, heads=h, head_dim=d, lse_out=lse)
    one = torch.empty_like(o)
    lse1 = torch.empty(h, lq, device=DEV)
    ops.attention(q, k, v, one, heads=h, head_dim=d, batch=1, lq=lq, q_bstride=0, l0=L, k0_bstride=0, lse=lse1)
    torch.cuda.synchronize()
    assert _rel(o, one) < 1e-5
    assert float((lse - lse1).abs().max()) < 1e-4


def _deq(q8, e):
    return q8.view(torch.float8_e4m3fn).double() * (2.0 ** int(e))


@pytest.mark.parametrize("fp8_v", [False, True], ids=["qk8", "qkv8"])
@pytest.mark.parametrize("bound", [False, True], ids=["scan", "static"])
@pytest.mark.parametrize("L", [43_968, 175_872], ids=["C3", "C5"])
def test_global_attention_fp8_production(ops, L, fp8_v, bound):
    """C5's fp8 path at full length with one power-of-two scale per tensor; a few outlier rows
    (x30) set amax, so the rest of q / k sit ~5 binades below it (the amax-driven
    scale at full length).  ``static``: the key_norm_max bound (the aggregator passes the qk-norm
    bound), which turns on the fixed-offset sweep in the q.k^T-only mode (waves whose rows' bound
    is > 100 above their tile-0 max, e.g. the x30 outlier, keep the per-tile max)."""
    q, k, v = _make(L, 11, spikes=(L - 101,))
    q[123] = (q[123].float() * 30).bfloat16()
    k[L // 3] = (k[L // 3].float() * 30).bfloat16()
    o = torch.empty(L, C, device=DEV, dtype=torch.bfloat16)
    ws = ops.Fp8Workspace()
    kb = float(k.float().view(-1, H, D).norm(dim=-1).max()) if bound else 0.0
    ops.attention_qk8(q, k, v, o, heads=H, batch=1, lq=L, q_bstride=0, l0=L, k0_bstride=0, ws=ws, fp8_v=fp8_v,
                      key_norm_max=kb)
    torch.cuda.synchronize()
    q8, k8, ex = ws.get(L, L, C, q.device)
    eq, ek, ev = (int(t) for t in ex.tolist())
    scale = D ** -0.5
    cfac = scale * math.log2(math.e)
    rows = _sample_rows(L, 256, L + 1).to(DEV)
    qd = _deq(q8[rows], eq) / cfac
    kd = _deq(k8, ek)
    vd = v.double()
    if fp8_v:
        vd = (v.float() * 2.0 ** -ev).to(torch.float8_e4m3fn).double() * 2.0 ** ev
    ref = _ref_rows(qd, kd, vd, scale)
    e_deq = _rel(o[rows].float(), ref)
    # and against the exact (bf16-operand) attention: the fp8 rounding itself.  e4m3 keeps a 2^-4
    # relative error per operand, so a score's absolute error grows with |score|: on this peaked
    # softmax (spike key ~12 nats above the rest, x30 outlier rows setting amax) it measured
    # 9.1e-2 rel-L2 for qk8 at C3 (the unit-scale inputs of test_fp8_gpu.py: <= 5e-2)
    e_exact = _rel(o[rows].float(), _ref_rows(q[rows], k, v, scale))
    print(f"fp8 {'qkv8' if fp8_v else 'qk8'} L={L}: vs dequantised {e_deq:.3e}, vs exact {e_exact:.3e}")
    assert e_deq < (3e-2 if fp8_v else 1e-2)
    assert e_exact < 0.15


def _padded(t, rows=64):
    """t with `rows` zero rows after it in memory (a runtime.Workspace buffer's padding)."""
    buf = torch.zeros(t.shape[0] + rows, *t.shape[1:], device=t.device, dtype=t.dtype)
    buf[:t.shape[0]] = t
    return buf[:t.shape[0]]


@pytest.mark.parametrize("tail", [False, True], ids=["compiled", "asm-seg"])
@pytest.mark.parametrize("nq,nsub", [(8, 8 * PP), (32, 32 * PP), (4, 32 * PP), (8, 32 * PP)],
                         ids=["C2", "C3", "C3-8rk", "C3-4rk"])
def test_reloc_attention_production(ops, nq, nsub, tail):
    """global_reloc (aggregator.py:672-741): every query frame attends to the shared anchor
    subsample (segment 0, batch stride 0) and to its own frame (segment 1); C3-8rk / C3-4rk are
    the per-rank shapes of the frame-sharded C3 forward (4 / 8 query frames).  asm-seg: readable
    rows past each segment (tail_readable, as the aggregator's workspace buffers) send the launch
    through the hand-scheduled sweep's two-segment / ragged-tail variant."""
    q, k, v = _make(nq * P, 3, spikes=(nq * P - 11,))
    ks, _, vs = _make(nsub, 4, spikes=(nsub - 3,))
    if tail:
        k, v, ks, vs = _padded(k), _padded(v), _padded(ks), _padded(vs)
    o = torch.empty(nq * P, C, device=DEV, dtype=torch.bfloat16)
    with ops.tuning(SR_ATTN_PIPE_SEG=int(tail)):  # the opt-in variant (sr_set_tuning)
        ops.attention(q, ks, vs, o, heads=H, head_dim=D, batch=nq, lq=P, q_bstride=P, l0=nsub, k0_bstride=0,
                      k1=k, v1=v, l1=P, k1_bstride=P, tail_readable=tail)
        # the library's dispatch: 256-row workgroups with the asm variant, or 128-row ones below 512
        # workgroups (the 4-query-frame rank shape)
        big = (P + 255) // 256 * H * nq >= 512
        assert ops.last_kernel() == (f"attn_bf16_kernel<4, 2, 1, {'true' if tail else 'false'}>" if big
                                     else "attn_bf16_kernel<2, 2, 1, false>")
    frames = sorted(set([0, nq - 1] + torch.randperm(nq, generator=torch.Generator().manual_seed(nq))[:6].tolist()))
    scale = D ** -0.5
    for j in frames:
        fr = slice(j * P, (j + 1) * P)
        rows = _sample_rows(P, 40, j).to(DEV)
        kk = torch.cat([ks, k[fr]])
        vv = torch.cat([vs, v[fr]])
        ref = _ref_rows(q[fr][rows], kk, vv, scale)
        assert _rel(o[fr][rows].float(), ref) < 1e-2, j


@pytest.mark.parametrize("nq", [8, 32], ids=["C2", "C3"])
def test_reloc_attention_split_production(ops, nq):
    """global_reloc as the aggregator's split (default; SR_RELOC_SPLIT=0 = one launch): every query row against the
    shared subsample's whole 64-key tiles as one long query set (the hand-scheduled sweep), each
    frame against the subsample's last partial tile + itself, merged by LSE with mixed layouts in
    the bf16 merge kernel; equal to the one-launch kernel and to fp64 on sampled rows."""
    nsub = 32 * PP
    q, k, v = _make(nq * P, 3, spikes=(nq * P - 11,))
    ks, _, vs = _make(nsub, 4, spikes=(nsub - 3, 100))
    rows, nf = nq * P, nsub // 64 * 64
    o_parts, lse_parts = ops.key_split_workspace(DEV, 2, rows, C, H, name="test_reloc_split")
    ops.attention(q, ks[:nf], vs[:nf], o_parts[:rows], heads=H, head_dim=D, batch=1, lq=rows, q_bstride=0, l0=nf,
                  k0_bstride=0, lse=lse_parts[0].view(-1))
    ops.attention(q, ks[nf:], vs[nf:], o_parts[rows:], heads=H, head_dim=D, batch=nq, lq=P, q_bstride=P,
                  l0=nsub - nf, k0_bstride=0, k1=k, v1=v, l1=P, k1_bstride=P, lse=lse_parts[1].view(-1))
    o = torch.empty(rows, C, device=DEV, dtype=torch.bfloat16)
    ops.attn_merge_n(o_parts, lse_parts, o, parts=2, rows=rows, heads=H, head_dim=D, seg_rows=[rows, P])
    one = torch.empty_like(o)
    ops.attention(q, ks, vs, one, heads=H, head_dim=D, batch=nq, lq=P, q_bstride=P, l0=nsub, k0_bstride=0,
                  k1=k, v1=v, l1=P, k1_bstride=P)
    # the aggregator's form: the second pass folds the first in (sr_attn_desc.merge_o) and writes the
    # union's LSE; the one-launch kernel's LSE is the reference for it
    om = torch.empty_like(o)
    lse_m = torch.empty(nq, H, P, device=DEV)
    ops.attention(q, ks[nf:], vs[nf:], om, heads=H, head_dim=D, batch=nq, lq=P, q_bstride=P, l0=nsub - nf,
                  k0_bstride=0, k1=k, v1=v, l1=P, k1_bstride=P, lse=lse_m.view(-1), merge_o=o_parts[:rows],
                  merge_lse=lse_parts[0])
    lse_one = torch.empty(nq, H, P, device=DEV)
    ops.attention(q, ks, vs, one, heads=H, head_dim=D, batch=nq, lq=P, q_bstride=P, l0=nsub, k0_bstride=0,
                  k1=k, v1=v, l1=P, k1_bstride=P, lse=lse_one.view(-1))
    torch.cuda.synchronize()
    assert _rel(o.float(), one.float()) < 1e-2
    assert _rel(om.float(), one.float()) < 1e-2
    assert _rel(om.float(), o.float()) < 5e-3  # same partials, the merge in fp32 either way
    assert float((lse_m - lse_one).abs().max()) < 1e-2
    scale = D ** -0.5
    for j in sorted({0, nq // 2, nq - 1}):
        fr = slice(j * P, (j + 1) * P)
        rws = _sample_rows(P, 40, j).to(DEV)
        ref = _ref_rows(q[fr][rws], torch.cat([ks, k[fr]]), torch.cat([vs, v[fr]]), scale)
        assert _rel(o[fr][rws].float(), ref) < 1e-2, j
        assert _rel(om[fr][rws].float(), ref) < 1e-2, j


@pytest.mark.parametrize("tail", [False, True], ids=["compiled", "asm-seg"])
def test_frame_attention_production(ops, tail):
    """frame / DINO stacks at C3: 64 frames x 1374 tokens, keys = own frame (asm-seg: the ragged
    last key tile staged whole from readable rows and masked in the hand-scheduled sweep)."""
    S = 64
    q, k, v = _make(S * P, 5, spikes=(S * P - 2,))
    if tail:
        k, v = _padded(k), _padded(v)
    o = torch.empty(S * P, C, device=DEV, dtype=torch.bfloat16)
    with ops.tuning(SR_ATTN_PIPE_SEG=int(tail)):
        ops.attention(q, k, v, o, heads=H, head_dim=D, batch=S, lq=P, q_bstride=P, l0=P, k0_bstride=P,
                      tail_readable=tail)
        assert ops.last_kernel() == f"attn_bf16_kernel<4, 2, 0, {'true' if tail else 'false'}>"
    scale = D ** -0.5
    for j in (0, 17, 40, S - 1):
        fr = slice(j * P, (j + 1) * P)
        rows = _sample_rows(P, 64, j).to(DEV)
        ref = _ref_rows(q[fr][rows], k[fr], v[fr], scale)
        assert _rel(o[fr][rows].float(), ref) < 1e-2, j


@pytest.mark.parametrize("S,L,static", [(16, P, True), (16, P, False), (40, 300, True), (5, P, False),
                                        (24, 777, True)],
                         ids=["16x1374", "16x1374-keyscan", "40x300", "5x1374-keyscan", "24x777"])
def test_frame_attention_shapes_lse(ops, S, L, static):
    """Frame launches of other sizes: ragged q- and key tiles, the static key bound and the
    per-frame key scan (DINO), a spike key forcing the running-max path in two frames, O and the
    log2-domain LSE the training backward reads, against fp64 on every frame's sampled rows
    (LSE: 3e-3 relative + 1e-2, the bf16 rounding of c*q)."""
    q, k, v = _make(S * L, 7 + S, spikes=(S * L - 5, L // 2))
    kn = 1.01 * float(k.float().view(-1, H, D).norm(dim=-1).max()) if static else 0.0
    o = torch.empty(S * L, C, device=DEV, dtype=torch.bfloat16)
    lse = torch.empty(S, H, L, device=DEV, dtype=torch.float32)
    ops.attention(q, k, v, o, heads=H, head_dim=D, batch=S, lq=L, q_bstride=L, l0=L, k0_bstride=L,
                  key_norm_max=kn, lse=lse)
    scale = D ** -0.5
    for j in range(S):
        fr = slice(j * L, (j + 1) * L)
        rows = _sample_rows(L, 24, j).to(DEV)
        ref = _ref_rows(q[fr][rows], k[fr], v[fr], scale)
        assert _rel(o[fr][rows].float(), ref) < 1e-2, j
        for h in (0, H - 1):
            c = slice(h * D, (h + 1) * D)
            sc = (q[fr][rows][:, c].double() @ k[fr][:, c].double().T) * scale
            ref_lse = torch.logsumexp(sc, -1) / math.log(2.0)
            # c*q enters the MFMAs rounded to bf16: scores (and so the LSE) carry ~2^-9 relative error
            err = (lse[j, h, rows].double() - ref_lse).abs() - 3e-3 * ref_lse.abs()
            assert float(err.max()) < 1e-2, (j, h)


def _qk_gain(rows, g, gen):
    """[rows, C] bf16 as the aggregator's qk-norm makes q / k (attention.py:49-50,78): per-head
    LayerNorm of a gaussian times w + b with w = g (1 + 0.02 n), b = 0.02 n -- the synthetic rule's
    affine scaled by the qk-gain g (trained q_norm / k_norm weights sit around 2-3).  Returns it and
    runtime.key_norm_bound's static bound sqrt(D) max|w| + |b| (x 1 + 2^-6)."""
    x = torch.randn(rows, H, D, device=DEV, generator=gen)
    x = (x - x.mean(-1, keepdim=True)) / x.std(-1, keepdim=True, unbiased=False)
    w = g * (1.0 + 0.02 * torch.randn(D, device=DEV, generator=gen))
    b = 0.02 * torch.randn(D, device=DEV, generator=gen)
    kb = (D ** 0.5 * float(w.abs().max()) + float(b.norm())) * (1.0 + 2.0 ** -6)
    return (x * w + b).reshape(rows, C).bfloat16(), kb


@pytest.mark.parametrize("g", [1.0, 2.0, 4.0, 8.0])
def test_global_attention_qk_gain(ops, g):
    """the hand-scheduled global sweep under trained-like qk-norm gains.  The
    Cauchy-Schwarz bound qb = c |q| k_bound grows as g^2 (~12 at g = 1, ~196 at g = 4); the sweep
    fixes m = max(0, qb - 64) per row, checked against the rows' max over the first three key tiles
    (sr_attn.hip PIPE_HI / PIPE_LO).  g <= 4: EVERY wave runs the hand-scheduled sweep
    (sr_attn_desc.sweep_stats), alone and paired with the reloc subsample pass; g = 8 (qb ~ 780,
    outside the window) falls to the compiled loop.  Each against fp64 on sampled rows, and the
    pair bit-identical to the two launches apart."""
    L, nf = 32 * P, 32 * PP // 64 * 64
    gen = torch.Generator(device=DEV).manual_seed(int(g * 10))
    q, _ = _qk_gain(L, g, gen)
    k, kb = _qk_gain(L, g, gen)
    v = torch.randn(L, C, device=DEV, generator=gen).bfloat16()
    qr, _ = _qk_gain(L, g, gen)
    ks, kbs = _qk_gain(nf, g, gen)
    vs = torch.randn(nf, C, device=DEV, generator=gen).bfloat16()
    st = torch.zeros(2, dtype=torch.int32, device=DEV)
    o = torch.empty(L, C, device=DEV, dtype=torch.bfloat16)
    ops.attention(q, k, v, o, heads=H, head_dim=D, batch=1, lq=L, q_bstride=0, l0=L, k0_bstride=0,
                  key_norm_max=kb, sweep_stats=st)
    sp = torch.zeros(2, dtype=torch.int32, device=DEV)
    og, orr = torch.empty_like(o), torch.empty_like(o)
    lse = torch.empty(H, L, device=DEV)
    ops.attention_pair(dict(q=q, k0=k, v0=v, o=og, lq=L, l0=L, key_norm_max=kb, sweep_stats=sp),
                       dict(q=qr, k0=ks, v0=vs, o=orr, lq=L, l0=nf, key_norm_max=kbs, lse=lse.view(-1),
                            sweep_stats=sp), heads=H, head_dim=D)
    or1 = torch.empty_like(o)
    lse1 = torch.empty_like(lse)
    ops.attention(qr, ks, vs, or1, heads=H, head_dim=D, batch=1, lq=L, q_bstride=0, l0=nf, k0_bstride=0,
                  key_norm_max=kbs, lse=lse1.view(-1))
    torch.cuda.synchronize()
    waves = (L + 63) // 64 * H  # waves with query rows: 64 rows each
    s1, s2 = st.tolist(), sp.tolist()
    print(f"qk-gain {g}: asm / compiled waves: global {s1}, pair {s2}")
    assert sum(s1) == waves and sum(s2) == 2 * waves
    if g <= 4.0:
        assert s1[1] == 0 and s2[1] == 0
    else:
        assert s1[1] > 0
    assert torch.equal(og, o) and torch.equal(orr, or1) and torch.equal(lse, lse1)
    scale = D ** -0.5
    # the kernels (asm and compiled alike) take c*q rounded to bf16 (c = scale*log2 e), a relative
    # error of 2^-9 on every score: at g = 8 the scores reach |s| ~ 300 (log2 domain), so the peaked
    # softmax moves by ~1.5e-2 against fp64 on the unscaled bf16 q (measured); 1e-2 up to g = 4
    tol = 1e-2 if g <= 4.0 else 3e-2
    for q_, k_, v_, o_ in ((q, k, v, o), (qr, ks, vs, orr)):
        rows = _sample_rows(L, 128, int(g)).to(DEV)
        ref = _ref_rows(q_[rows], k_, v_, scale)
        assert _rel(o_[rows].float(), ref) < tol
    # the second problem's LSE (log2 domain), as test_attention_pair
    rws = _sample_rows(L, 32, 3).to(DEV)
    for h in (0, H - 1):
        c = slice(h * D, (h + 1) * D)
        sc = (qr[rws][:, c].double() @ ks[:, c].double().T) * scale
        l2 = torch.logsumexp(sc, -1) / math.log(2.0)
        assert float(((lse[h, rws].double() - l2).abs() - 3e-3 * l2.abs()).max()) < 3e-2


def _vt_ref(v, L, heads):
    """sr_vt_tiles' layout in torch: [heads][ceil(L/64)][64 d][64 slots], slot 32kb + 16s2 + 8h + j
    holding key 32kb + 16s2 + 8(j >> 2) + 4h + (j & 3) of the tile (zero past L)."""
    nt = (L + 63) // 64
    vp = torch.zeros(nt * 64, heads * D, dtype=v.dtype, device=v.device)
    vp[:L] = v[:L, :heads * D]
    p = torch.arange(64)
    j = p & 7
    key = (p & 48) + 8 * (j >> 2) + 4 * ((p >> 3) & 1) + (j & 3)
    t = vp.view(nt, 64, heads, D)[:, key.to(v.device)]          # [tile][slot][head][d]
    return t.permute(2, 0, 3, 1).contiguous()                    # [head][tile][d][slot]


@pytest.mark.parametrize("case", ["C3", "padded", "gain8"])
def test_attention_pair_vt(ops, case):
    """sr_attention_pair_vt (V^T tiles from sr_vt_tiles, one ds_read_b128 per P.V fragment) is
    bit-identical to sr_attention_pair, on the hand-scheduled sweep (C3, 'padded': 3 heads and a
    padded first problem) and on the compiled fallback loop ('gain8': qk-norm gain 8 puts the rows
    outside the fixed-offset window, sweep_stats counts compiled waves).  The tiles match the
    layout built in torch (ragged L included)."""
    if case == "C3":
        heads, La, rows, nk = H, 32 * P, 32 * P, 32 * PP // 64 * 64
        qg, kg, vg = _make(La, 11, spikes=(La - 5, 77))
        qr, _, _ = _make(rows, 12)
        _, ks, vs = _make(nk, 13, spikes=(nk - 1,))
        kbg, kbr = _kbound(kg, heads), _kbound(ks, heads)
    elif case == "padded":
        heads, La, rows, nk = 3, 21 * 256 - 128, 9 * 256 + 7, 40 * 64
        g = torch.Generator(device=DEV).manual_seed(5)
        mk = lambda n: (torch.randn(n, heads * D, device=DEV, generator=g) * 0.5).bfloat16()  # noqa: E731
        qg, kg, vg, qr, ks, vs = mk(La), mk(La), mk(La), mk(rows), mk(nk), mk(nk)
        kbg, kbr = _kbound(kg, heads), _kbound(ks, heads)
    else:
        heads, La, nk = H, 16 * P, 16 * PP // 64 * 64
        La = La // 64 * 64
        rows = La
        gen = torch.Generator(device=DEV).manual_seed(80)
        qg, _ = _qk_gain(La, 8.0, gen)
        kg, kbg = _qk_gain(La, 8.0, gen)
        vg = torch.randn(La, C, device=DEV, generator=gen).bfloat16()
        qr, _ = _qk_gain(rows, 8.0, gen)
        ks, kbr = _qk_gain(nk, 8.0, gen)
        vs = torch.randn(nk, C, device=DEV, generator=gen).bfloat16()
    cols = heads * D
    vtg = torch.empty(ops.vt_tile_shape(La, heads), dtype=torch.bfloat16, device=DEV)
    vtr = torch.empty(ops.vt_tile_shape(nk, heads), dtype=torch.bfloat16, device=DEV)
    ops.vt_tiles(vg, La, heads, vtg)
    ops.vt_tiles(vs, nk, heads, vtr)
    outs = []
    for vt in (None, (vtg, vtr)):
        og, orr = (torch.empty(n, cols, device=DEV, dtype=torch.bfloat16) for n in (La, rows))
        lse = torch.empty(heads, rows, device=DEV)
        st = torch.zeros(2, dtype=torch.int32, device=DEV)
        a = dict(q=qg, k0=kg, v0=vg, o=og, lq=La, l0=La, key_norm_max=kbg, sweep_stats=st)
        b = dict(q=qr, k0=ks, v0=vs, o=orr, lq=rows, l0=nk, key_norm_max=kbr, lse=lse.view(-1), sweep_stats=st)
        if vt is not None:
            a["vt"], b["vt"] = vt
        ops.attention_pair(a, b, heads=heads, head_dim=D)
        torch.cuda.synchronize()
        outs.append((og, orr, lse, st.tolist()))
    print(f"pair_vt {case}: asm / compiled waves {outs[1][3]}")
    assert outs[0][3] == outs[1][3]
    if case == "gain8":
        assert outs[1][3][1] > 0
    else:
        assert outs[1][3][1] == 0
    for x, y in zip(outs[0][:3], outs[1][:3]):
        assert torch.equal(x, y)
    assert torch.equal(vtg.view(heads, -1, 64, 64), _vt_ref(vg, La, heads))
    # a ragged L (keys past L zero) and a strided V (columns of a wider row)
    Lr = 1000
    wide = torch.randn(Lr, 3 * cols, device=DEV).bfloat16()
    vt_r = torch.full(ops.vt_tile_shape(Lr, heads), 7.0, dtype=torch.bfloat16, device=DEV)
    ops.vt_tiles(wide[:, cols:2 * cols], Lr, heads, vt_r)
    assert torch.equal(vt_r.view(heads, -1, 64, 64), _vt_ref(wide[:, cols:2 * cols], Lr, heads))


def test_attention_dma_base_bit31(ops):
    """The round-3 fault's cause (readfirstlane returns int, and the widened low
    word of the LDS-DMA base sign-extended into the high word when bit 31 was set; fixed at
    sr_attn.hip's sp_lo / sp_hi): q / k / v placed so that every DMA base address the asm sweep
    forms has bit 31 of its low word set.  The global attention and the pair launch there are
    bit-identical to the same data at an ordinary address."""
    L, nf = 171 * 64, 8 * PP // 64 * 64  # whole key tiles: the pair and the plain asm variant
    q, k, v = _make(L, 21, spikes=(L - 9,))
    ks, _, vs = _make(nf, 22)
    kb, kbs = _kbound(k), _kbound(ks)
    slab = 3 * L * C * 2 + 2 * nf * C * 2
    big = torch.empty(slab + (1 << 32) + 4096, dtype=torch.uint8, device=DEV)
    base = big.data_ptr()
    off = ((0x90000000 - (base & 0xFFFFFFFF)) % (1 << 32) + 255) // 256 * 256
    region = big[off:off + slab]
    assert ((base + off) & 0xFFFFFFFF) >= 0x80000000 and ((base + off + slab) & 0xFFFFFFFF) >= 0x80000000

    def at(t, start):
        n = t.numel() * 2
        dst = region[start:start + n].view(torch.bfloat16).view(t.shape)
        dst.copy_(t)
        return dst, start + n
    s = 0
    q2, s = at(q, s)
    k2, s = at(k, s)
    v2, s = at(v, s)
    ks2, s = at(ks, s)
    vs2, s = at(vs, s)
    outs = []
    for (qq, kk, vv, kks, vvs) in ((q, k, v, ks, vs), (q2, k2, v2, ks2, vs2)):
        o = torch.empty(L, C, device=DEV, dtype=torch.bfloat16)
        og, orr = torch.empty_like(o), torch.empty_like(o)
        st = torch.zeros(2, dtype=torch.int32, device=DEV)
        ops.attention(qq, kk, vv, o, heads=H, head_dim=D, batch=1, lq=L, q_bstride=0, l0=L, k0_bstride=0,
                      key_norm_max=kb, sweep_stats=st)
        ops.attention_pair(dict(q=qq, k0=kk, v0=vv, o=og, lq=L, l0=L, key_norm_max=kb),
                           dict(q=qq, k0=kks, v0=vvs, o=orr, lq=L, l0=nf, key_norm_max=kbs), heads=H, head_dim=D)
        torch.cuda.synchronize()
        assert st.tolist()[1] == 0  # every wave on the hand-scheduled sweep
        outs.append((o, og, orr))
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    del big


def _qk_gain_shared(rows, g, gen, u, spread):
    """_qk_gain's rule on inputs u + spread * n (a direction u shared by every row): the keys of a
    real forward cluster like this, so the rows' scores sit far below the 2-norm bound c|q||k|."""
    x = u + spread * torch.randn(rows, H, D, device=DEV, generator=gen)
    x = (x - x.mean(-1, keepdim=True)) / x.std(-1, keepdim=True, unbiased=False)
    w = g * (1.0 + 0.02 * torch.randn(D, device=DEV, generator=gen))
    b = 0.02 * torch.randn(D, device=DEV, generator=gen)
    kb = (D ** 0.5 * float(w.abs().max()) + float(b.norm())) * (1.0 + 2.0 ** -6)
    return (x * w + b).reshape(rows, C).bfloat16(), kb


@pytest.mark.parametrize("g", [2.0, 4.0])
def test_global_attention_key_box(ops, g):
    """The per-dimension key box (sr_attention_key_box, sr_attn_desc.key_box): keys clustered
    around one direction, queries spread, qk-gain g.  With the 2-norm bound alone (query_norm_max
    0) the rows whose queries point away from the keys' direction lie > 174 below it and their waves
    fall to the compiled loop (at g = 4); with query_norm_max the launch computes the box, whose
    bound sits within the window, and every wave stays on the hand-scheduled sweep, alone and paired.
    Both against fp64 on sampled rows; the box itself bit-exact against torch's amax / amin."""
    L, nf = 32 * P, 32 * PP // 64 * 64
    gen = torch.Generator(device=DEV).manual_seed(int(g * 100))
    u = torch.randn(1, H, D, device=DEV, generator=gen)
    q, qn = _qk_gain(L, g, gen)
    k, kb = _qk_gain_shared(L, g, gen, u, 0.05)
    v = torch.randn(L, C, device=DEV, generator=gen).bfloat16()
    ks, kbs = _qk_gain_shared(nf, g, gen, u, 0.05)
    vs = torch.randn(nf, C, device=DEV, generator=gen).bfloat16()
    box = torch.empty(H, 2, D, device=DEV)
    lib = ops._lib.load()
    sc = torch.empty(lib.sr_attention_key_box_scratch(L, 1, H), device=DEV)
    assert lib.sr_attention_key_box(ops._stream(k), k.data_ptr(), C, L, 0, 1, H, box.data_ptr(), None,
                                    sc.data_ptr()) == 0
    kh = k.float().view(L, H, D)
    assert torch.equal(box[:, 0], kh.amax(0)) and torch.equal(box[:, 1], kh.amin(0))
    outs = {}
    for qnm in (0.0, qn):
        st = torch.zeros(2, dtype=torch.int32, device=DEV)
        o = torch.empty(L, C, device=DEV, dtype=torch.bfloat16)
        ops.attention(q, k, v, o, heads=H, head_dim=D, batch=1, lq=L, q_bstride=0, l0=L, k0_bstride=0,
                      key_norm_max=kb, query_norm_max=qnm, sweep_stats=st)
        sp = torch.zeros(2, dtype=torch.int32, device=DEV)
        og, orr = torch.empty_like(o), torch.empty_like(o)
        ops.attention_pair(dict(q=q, k0=k, v0=v, o=og, lq=L, l0=L, key_norm_max=kb, query_norm_max=qnm,
                                sweep_stats=sp),
                           dict(q=q, k0=ks, v0=vs, o=orr, lq=L, l0=nf, key_norm_max=kbs, query_norm_max=qnm,
                                sweep_stats=sp), heads=H, head_dim=D)
        torch.cuda.synchronize()
        print(f"qk-gain {g}, query_norm_max {qnm:.1f}: asm / compiled waves: global {st.tolist()}, "
              f"pair {sp.tolist()}")
        outs[qnm] = (st.tolist(), sp.tolist(), o, og, orr)
    waves = (L + 63) // 64 * H
    s_cs, p_cs = outs[0.0][:2]
    s_bx, p_bx = outs[qn][:2]
    assert sum(s_bx) == waves and sum(p_bx) == 2 * waves
    assert s_bx[1] == 0 and p_bx[1] == 0
    if g >= 4.0:
        assert s_cs[1] > 0  # the 2-norm bound alone leaves the window
    scale = D ** -0.5
    rows = _sample_rows(L, 128, int(g)).to(DEV)
    ref = _ref_rows(q[rows], k, v, scale)
    refs = _ref_rows(q[rows], ks, vs, scale)
    for qnm in (0.0, qn):
        _, _, o, og, orr = outs[qnm]
        assert _rel(o[rows].float(), ref) < 1e-2
        assert torch.equal(og, o)
        assert _rel(orr[rows].float(), refs) < 1e-2


@pytest.mark.parametrize("vscale", [1.0, 2.0 ** 40], ids=["v1", "v2e40"])
def test_global_attention_value_window(ops, vscale):
    """The value box (sr_attn_desc.value_box): qk-gain 4.5 on LayerNorm'd random q / k puts every
    wave's gap between its bound and its max over the first three key tiles at ~195 > 174 (the
    default 2^64 / 2^-110 window), so the 2-norm window alone sends every wave to the compiled loop.
    With max|v| known the upper side widens to 125 - ceil(log2 L) - ceil(log2 max|v|) = 106 -> 100
    (|v| ~ 4): every wave runs the hand-scheduled sweep.  V scaled by 2^40 narrows it to 66 (a
    176-wide window): most waves fall back, correctly.  (With the boxes the launch also scans the
    keys' actual max norm, ~5 % below the static bound here.)  Against fp64 on sampled rows."""
    g, L = 4.5, 32 * P
    gen = torch.Generator(device=DEV).manual_seed(45)
    q, qn = _qk_gain(L, g, gen)
    k, kb = _qk_gain(L, g, gen)
    v = (torch.randn(L, C, device=DEV, generator=gen) * vscale).bfloat16()
    res = {}
    for qnm in (0.0, qn):
        st = torch.zeros(2, dtype=torch.int32, device=DEV)
        o = torch.empty(L, C, device=DEV, dtype=torch.bfloat16)
        ops.attention(q, k, v, o, heads=H, head_dim=D, batch=1, lq=L, q_bstride=0, l0=L, k0_bstride=0,
                      key_norm_max=kb, query_norm_max=qnm, sweep_stats=st)
        torch.cuda.synchronize()
        print(f"v x {vscale:g}, query_norm_max {qnm:.1f}: asm / compiled waves {st.tolist()}")
        res[qnm] = (st.tolist(), o)
    waves = (L + 63) // 64 * H
    assert res[0.0][0] == [0, waves]
    if vscale == 1.0:
        assert res[qn][0] == [waves, 0]
    else:  # only the waves whose gap fits the narrower window stay on the sweep
        assert res[qn][0][1] > waves // 2
    rows = _sample_rows(L, 128, 45).to(DEV)
    ref = _ref_rows(q[rows], k, v, D ** -0.5)
    for qnm in (0.0, qn):
        err = _rel(res[qnm][1][rows].float(), ref)
        print(f"rel err vs fp64 (query_norm_max {qnm:.1f}): {err:.2e}")
        assert err < 1.5e-2  # c*q in bf16 at |s| ~ 300: as test_global_attention_qk_gain


@pytest.mark.parametrize("tail", [False, True], ids=["compiled", "asm_seg"])
def test_global_attention_key_split_boxes(ops, tail):
    """The data-derived bounds on the key-split path (attention_partials, one box / norm / value box
    instance per key chunk): a G = 8 rank's query slice (5,496 rows) at qk-gain 4 against the C3
    keys clustered around one direction, with (query_norm_max set) and without the boxes, each
    against fp64.  ``tail``: the chunks' ragged tails readable (padded key buffer), so the chunks
    may take the hand-scheduled _SEG sweep."""
    g, L = 4.0, 32 * P
    lq = 4 * P
    gen = torch.Generator(device=DEV).manual_seed(404)
    u = torch.randn(1, H, D, device=DEV, generator=gen)
    q, qn = _qk_gain(lq, g, gen)
    k, kb = _qk_gain_shared(L, g, gen, u, 0.05)
    v = torch.randn(L, C, device=DEV, generator=gen).bfloat16()
    if tail:
        k, v = _padded(k), _padded(v)
    parts = ops.key_split_parts(dtype=torch.bfloat16, batch=1, lq=lq, heads=H, l0=L, l1=0, mask_mode=0)
    assert parts > 1
    rows = _sample_rows(lq, 128, 404).to(DEV)
    ref = _ref_rows(q[rows], k[:L], v[:L], D ** -0.5)
    outs = []
    for qnm in (0.0, qn):
        o = torch.empty(lq, C, device=DEV, dtype=torch.bfloat16)
        ops.attention(q, k, v, o, heads=H, head_dim=D, batch=1, lq=lq, q_bstride=0, l0=L, k0_bstride=0,
                      key_norm_max=kb, query_norm_max=qnm, tail_readable=tail)
        torch.cuda.synchronize()
        err = _rel(o[rows].float(), ref)
        print(f"key split S={parts}, tail {tail}, query_norm_max {qnm:.1f}: rel {err:.2e}")
        assert err < 1e-2
        outs.append(o)
    assert _rel(outs[1].float(), outs[0].float()) < 1e-2


@pytest.mark.parametrize("tail", [False, True], ids=["compiled", "asm-seg"])
def test_reloc_attention_two_segment_boxes(ops, tail):
    """The data-derived bounds on a two-segment launch (global_reloc at qk-gain 4): the shared
    subsample (segment 0, one box / norm / value-box instance) and each query frame's own keys
    (segment 1, one instance per frame, at kb_n0 + item), both clustered around one direction so
    that the boxes change the bound.  With and without them, against fp64 per frame."""
    g, nq, nsub = 4.0, 8, 8 * PP
    gen = torch.Generator(device=DEV).manual_seed(77)
    u = torch.randn(1, H, D, device=DEV, generator=gen)
    q, qn = _qk_gain(nq * P, g, gen)
    k, kb = _qk_gain_shared(nq * P, g, gen, u, 0.05)
    ks, kbs = _qk_gain_shared(nsub, g, gen, u, 0.05)
    v = torch.randn(nq * P, C, device=DEV, generator=gen).bfloat16()
    vs = torch.randn(nsub, C, device=DEV, generator=gen).bfloat16()
    if tail:
        k, v, ks, vs = _padded(k), _padded(v), _padded(ks), _padded(vs)
    kbound = max(kb, kbs)
    outs = []
    for qnm in (0.0, qn):
        o = torch.empty(nq * P, C, device=DEV, dtype=torch.bfloat16)
        with ops.tuning(SR_ATTN_PIPE_SEG=int(tail)):
            ops.attention(q, ks, vs, o, heads=H, head_dim=D, batch=nq, lq=P, q_bstride=P, l0=nsub, k0_bstride=0,
                          k1=k, v1=v, l1=P, k1_bstride=P, tail_readable=tail, key_norm_max=kbound,
                          query_norm_max=qnm)
        torch.cuda.synchronize()
        outs.append(o)
    scale = D ** -0.5
    for j in (0, 3, nq - 1):
        fr = slice(j * P, (j + 1) * P)
        rows = _sample_rows(P, 40, j).to(DEV)
        ref = _ref_rows(q[fr][rows], torch.cat([ks, k[fr]]), torch.cat([vs, v[fr]]), scale)
        for o in outs:
            assert _rel(o[fr][rows].float(), ref) < 1e-2, j
    assert _rel(outs[1].float(), outs[0].float()) < 1e-2


def test_global_attention_scan_boxes(ops):
    """Key-scan launches (no static key bound: the training forward) of one long query set attach
    the key and value boxes themselves (ops._attach_scan_boxes): at qk-gain 4.5 on LayerNorm'd random
    q / k every wave then runs the hand-scheduled sweep, where the scanned 2-norm window alone sends
    most waves to the compiled loop.  Both against fp64."""
    g, L = 4.5, 32 * P
    gen = torch.Generator(device=DEV).manual_seed(450)
    q, _ = _qk_gain(L, g, gen)
    k, _ = _qk_gain(L, g, gen)
    v = torch.randn(L, C, device=DEV, generator=gen).bfloat16()
    rows = _sample_rows(L, 128, 450).to(DEV)
    ref = _ref_rows(q[rows], k, v, D ** -0.5)
    waves = (L + 63) // 64 * H
    saved = ops._KEY_BOX
    try:
        for mode in ("0", "auto"):
            ops._KEY_BOX = mode
            st = torch.zeros(2, dtype=torch.int32, device=DEV)
            o = torch.empty(L, C, device=DEV, dtype=torch.bfloat16)
            ops.attention(q, k, v, o, heads=H, head_dim=D, batch=1, lq=L, q_bstride=0, l0=L, k0_bstride=0,
                          sweep_stats=st)
            torch.cuda.synchronize()
            err = _rel(o[rows].float(), ref)
            print(f"scan mode, SR_ATTN_KEY_BOX={mode}: waves {st.tolist()}, rel {err:.2e}")
            # without the boxes the scanned max |k| (tighter than the static bound) keeps a few waves
            # (measured 207 of 10,992) inside the 174-wide window
            assert st.tolist() == [waves, 0] if mode == "auto" else st.tolist()[1] > waves // 2
            assert err < 1.5e-2
    finally:
        ops._KEY_BOX = saved


@pytest.mark.parametrize("vexp", [0, -14], ids=["v1", "v2e-14"])
def test_attention_window_low_edge(ops, vexp):
    """ADVICE r4 (FIX_LO = 110): rows whose fixed offset m = max(0, qb - 64) sits 76-106 (log2) above
    their true score max, so the row's largest P is down to ~2^-106 (the window allows 2^-110), with
    V of order 1 and of order 2^-14 (every P.V product of the top keys >= 2^-121 stays a normal fp32).
    Construction (CPU generator, checked here): every query of a head points along one direction u
    with c|q||k| = 400; the first tile's keys make cosines 0.5-0.6 with u (the row max, inside the
    first three tiles the window is checked on); the rest are random (>= 33 below).  Every wave
    stays on the hand-scheduled sweep, and the result matches fp64 on sampled rows.  (Below
    |v| ~ 2^-16 at the window's very edge the P.V products would reach fp32 denormals.)"""
    L = 8192
    c = D ** -0.5 * LOG2E
    g = torch.Generator().manual_seed(101)
    u = torch.randn(H, D, generator=g)
    u = u / u.norm(dim=-1, keepdim=True)
    k = torch.randn(L, H, D, generator=g)
    w = torch.randn(64, H, D, generator=g)
    w = w - (w * u[None]).sum(-1, keepdim=True) * u[None]
    w = w / w.norm(dim=-1, keepdim=True)
    cs = torch.linspace(0.5, 0.6, 64)[:, None, None]
    k[:64] = cs * u[None] + torch.sqrt(1 - cs ** 2) * w
    k = (k * (8.0 / k.norm(dim=-1, keepdim=True))).reshape(L, C).bfloat16().to(DEV)
    q = u[None] + 0.02 * torch.randn(L, H, D, generator=g)
    q = q * (400.0 / (c * 8.0) / q.norm(dim=-1, keepdim=True))
    qs = (q * c).reshape(L, C).bfloat16().to(DEV)
    v = (torch.randn(L, C, generator=g) * 2.0 ** vexp).bfloat16().to(DEV)
    kb = _kbound(k)
    st = torch.zeros(2, dtype=torch.int32, device=DEV)
    o = torch.empty(L, C, device=DEV, dtype=torch.bfloat16)
    ops.attention(qs, k, v, o, heads=H, head_dim=D, batch=1, lq=L, q_bstride=0, l0=L, k0_bstride=0, key_norm_max=kb,
                  sweep_stats=st, q_scaled=True)
    torch.cuda.synchronize()
    rows = _sample_rows(L, 128, 5).to(DEV)
    s = torch.einsum("qhd,khd->hqk", qs[rows].view(-1, H, D).double(), k.view(-1, H, D).double())  # log2 domain
    m = (qs[rows].view(-1, H, D).double().norm(dim=-1).T * kb - 64.0).clamp_min(0)
    gap = m - s.amax(-1)
    e = _rel(o[rows].float(), _ref_rows(qs[rows], k, v, LN2))
    print(f"|v| ~ 2^{vexp}: offset above the true max {float(gap.min()):.1f} .. {float(gap.max()):.1f} (log2), "
          f"asm / compiled waves {st.tolist()}, rel vs fp64 {e:.2e}")
    assert float(gap.max()) > 95.0  # rows really sit near the window's low edge
    assert st.tolist()[1] == 0 and st.tolist()[0] == L // 64 * H
    assert e < 1e-2


@pytest.mark.parametrize("batch,L,heads", [(64, 1374, 16), (3, 261, 6), (1, 4099, 16), (5, 7, 2)])
def test_attention_key_scan(ops, batch, L, heads):
    """The launch's own key scan (no static bound: DINO's blocks, key_norm_max = 0): sr_attention
    fills key_bound with each (instance, head)'s max |k|^2 before the sweep (key_norm_max_kernel,
    4 rows' loads in flight per thread, a plain loop for the rest) -- against torch on the same
    bf16 keys, for row counts that leave every remainder of the unrolled loop."""
    g = torch.Generator(device="cpu").manual_seed(batch * 1000 + L)
    Cw = heads * D
    qkv = (torch.randn(batch * L, 3 * Cw, generator=g) * torch.linspace(0.5, 2.0, 3 * Cw)).bfloat16().to(DEV)
    o = torch.empty(batch * L, Cw, device=DEV, dtype=torch.bfloat16)
    ops.attention(qkv[:, :Cw], qkv[:, Cw:2 * Cw], qkv[:, 2 * Cw:], o, heads=heads, head_dim=D, batch=batch, lq=L,
                  q_bstride=L, l0=L, k0_bstride=L)
    torch.cuda.synchronize()
    kb = ops._train_ws(qkv.device, "attn_key_bound", batch * heads)[:batch * heads].view(batch, heads)
    ref = (qkv[:, Cw:2 * Cw].float().view(batch, L, heads, D) ** 2).sum(-1).amax(1)
    err = float(((kb - ref).abs() / ref).max())
    print(f"key scan batch={batch} L={L} heads={heads}: max rel {err:.2e}")
    assert err < 1e-6
