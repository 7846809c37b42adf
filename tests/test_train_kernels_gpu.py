"""Training-step kernels against torch fp32 statements of the same op on
the same (bf16-rounded) inputs, through the C ABI: weight-gradient GEMM, the backward GEMM
epilogues (F32, GELU_BWD, saved pre-activations), column sums, LayerNorm backward, qk-norm +
RoPE backward, cast, the non-finite check and the Adam step.

Tolerances: fp32 accumulation of bf16 products -> 1e-5 rel-L2 where the inputs are bf16 and
the output fp32 (wgrad, F32 epilogue, colsum); bf16 outputs 8e-3; LayerNorm / qk backward
in fp32 1e-5 (fp32 dy) or 8e-3 (bf16 outputs); Adam 1e-6."""

import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


@pytest.fixture(scope="module")
def ops():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from sailrecon_amd import ops as _ops
    return _ops


def L():
    from sailrecon_amd import _lib
    return _lib


# N, K multiples of 256 run the 256 x 256 kernel (wgrad256_kernel), the others the 128 x 128 one
@pytest.mark.parametrize("M,N,K,splits", [(64, 128, 128, 1), (1000, 256, 384, 1), (4397, 384, 256, 3),
                                          (43968 // 8, 1024, 1024, None), (130, 3072, 128, 2),
                                          (4397, 512, 256, 3), (200, 256, 256, 1), (21984, 3072, 1024, None),
                                          (43968, 1024, 4096, None)])
def test_gemm_wgrad(ops, M, N, K, splits):
    torch.manual_seed(0)
    dy = torch.randn(M, N, device=DEV).bfloat16()
    x = torch.randn(M, K, device=DEV).bfloat16()
    ref = dy.float().t() @ x.float()
    dw = torch.empty(N, K, device=DEV)
    ops.gemm_wgrad(dy, x, dw, splits=splits)
    assert rel(dw, ref) < 1e-5


@pytest.mark.parametrize("K", [128, 256])
def test_gemm_wgrad_strided_accumulate_rowscale_rowdot(ops, K):
    """Row-strided operands (column slices of wider buffers), accumulate, per-row scale
    (LayerScale gamma folded into dW) and rowdot (the gamma gradient)."""
    torch.manual_seed(1)
    M, N = 777, 256
    big_dy = torch.randn(M, N + 128, device=DEV).bfloat16()
    big_x = torch.randn(M, 3 * K, device=DEV).bfloat16()
    dy, x = big_dy[:, 128:], big_x[:, K:2 * K]
    dw0 = torch.randn(N, K, device=DEV)
    dw = dw0.clone()
    gamma = torch.randn(N, device=DEV)
    wdot = torch.randn(N, K, device=DEV)
    rowdot = torch.randn(N, device=DEV)
    rd0 = rowdot.clone()
    ops.gemm_wgrad(dy, x, dw, accumulate=True, rowscale=gamma, wdot=wdot, rowdot=rowdot, splits=4)
    G = dy.float().t() @ x.float()
    assert rel(dw, dw0 + gamma[:, None] * G) < 1e-5
    assert rel(rowdot - rd0, (wdot * G).sum(1)) < 1e-5


@pytest.mark.parametrize("M0, M1, N, K", [(21984, 21984, 1024, 4096), (21984, 4397, 1024, 1024),
                                          (777, 1300, 256, 512)])
def test_gemm_wgrad_pair(ops, M0, M1, N, K):
    """sr_gemm_wgrad_pair (the layer's reloc and global blocks' weight grads in one launch, as
    train.engine.block_bwd_multi runs them): per problem bit-identical to sr_gemm_wgrad with the
    same slices, with accumulate / rowscale / rowdot on one problem and not the other; and within
    fp32 rounding of dy^T x."""
    torch.manual_seed(4)
    probs, refs = [], []
    for i, M in enumerate((M0, M1)):
        dy = torch.randn(M, N, device=DEV).bfloat16()
        x = torch.randn(M, K, device=DEV).bfloat16()
        dw0 = torch.randn(N, K, device=DEV)
        p = dict(dy=dy, x=x, dw=dw0.clone())
        if i == 0:
            p.update(accumulate=True, rowscale=torch.randn(N, device=DEV), wdot=torch.randn(N, K, device=DEV),
                     rowdot=torch.zeros(N, device=DEV))
        probs.append(p)
        refs.append(dict(p, dw=dw0.clone(), rowdot=None if i else torch.zeros(N, device=DEV)))
    sp = ops.wgrad_pair_splits(M0, M1, N, K) or (3, 5)
    ops.gemm_wgrad_pair(probs, sp)
    for r, s in zip(refs, sp):
        ops.gemm_wgrad(r["dy"], r["x"], r["dw"], accumulate=r.get("accumulate", False), rowscale=r.get("rowscale"),
                       wdot=r.get("wdot"), rowdot=r.get("rowdot"), splits=s)
    torch.cuda.synchronize()
    for i, (p, r) in enumerate(zip(probs, refs)):
        assert torch.equal(p["dw"], r["dw"])
        G = p["dy"].float().t() @ p["x"].float()
        if i == 0:
            assert torch.equal(p["rowdot"], r["rowdot"])
            assert rel(p["rowdot"], (p["wdot"] * G).sum(1)) < 1e-5
        else:
            assert rel(p["dw"], G) < 1e-5


def test_gemm_f32_and_gelu_bwd_epilogues(ops):
    torch.manual_seed(2)
    lib = L()
    for M, N, K in ((300, 256, 128), (33000, 1024, 64)):  # 128x128 and 256x256 (>= 512 tiles) kernels
        a = torch.randn(M, K, device=DEV).bfloat16()
        w = (torch.randn(N, K, device=DEV) / 8).bfloat16()
        acc = a.float() @ w.float().t()
        out = torch.empty(M, N, device=DEV)
        bias = torch.randn(N, device=DEV)
        ops.gemm(a, w, out, lib.SR_EPI_F32, bias=bias)
        assert rel(out, acc + bias) < 1e-5
        u = torch.randn(M, N, device=DEV).bfloat16()
        dh = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        ops.gemm(a, w, dh, lib.SR_EPI_GELU_BWD, aux=u)
        uf = u.float()
        gprime = 0.5 * (1 + torch.erf(uf / math.sqrt(2))) + uf * torch.exp(-0.5 * uf * uf) / math.sqrt(2 * math.pi)
        assert rel(dh.float(), acc * gprime) < 8e-3


def test_gemm_saves_preactivation(ops):
    """Training forward: BIAS_GELU stores u = acc + bias; QKV stores the pre-norm q|k|v."""
    from sailrecon_amd.layers.rope import RotaryPositionEmbedding2D
    torch.manual_seed(3)
    lib = L()
    M, C, D = 21 * 40, 256, 64
    a = torch.randn(M, C, device=DEV).bfloat16()
    w = (torch.randn(4 * C, C, device=DEV) / 16).bfloat16()
    b = torch.randn(4 * C, device=DEV)
    h = torch.empty(M, 4 * C, device=DEV, dtype=torch.bfloat16)
    u = torch.empty_like(h)
    ops.gemm(a, w, h, lib.SR_EPI_BIAS_GELU, bias=b, aux=u)
    y = a.float() @ w.float().t() + b
    assert rel(u.float(), y) < 8e-3
    assert rel(h.float(), F.gelu(y)) < 8e-3
    wq = w[:3 * C].contiguous()
    raw = torch.empty(M, 3 * C, device=DEV, dtype=torch.bfloat16)
    out = torch.empty_like(raw)
    rope = RotaryPositionEmbedding2D(100).tables(D, 5, DEV)
    epi = dict(embed_dim=C, head_dim=D, qk_eps=1e-5, qn_w=torch.randn(D, device=DEV), qn_b=torch.randn(D, device=DEV),
               kn_w=torch.randn(D, device=DEV), kn_b=torch.randn(D, device=DEV), rope_cos=rope[0], rope_sin=rope[1],
               tokens_per_frame=21, patch_start=5, grid_w=4, pos_row_base=0)
    ops.gemm(a, wq, out, lib.SR_EPI_QKV, bias=b[:3 * C], qkv=epi, aux=raw)
    assert rel(raw.float(), y[:, :3 * C]) < 8e-3
    assert rel(out[:, 2 * C:].float(), y[:, 2 * C:3 * C]) < 8e-3


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("M,N", [(1, 5 * 1024), (31, 1369 * 64), (43968, 1024), (777, 4096)])
def test_colsum(ops, dtype, M, N):
    torch.manual_seed(4)
    big = torch.randn(M, N + 8, device=DEV).to(dtype)
    x = big[:, 4:N + 4]
    out = torch.randn(N, device=DEV)
    o0 = out.clone()
    ops.colsum(x, out, accumulate=True, scale=0.5)
    assert rel(out - o0, 0.5 * x.float().sum(0)) < 1e-5


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("M,N", [(31, 1024), (43968, 1024), (777, 4096)])
def test_colsum_fma(ops, dtype, M, N):
    """sr_colsum_fma (the LayerScale residual's bias / gamma grads in the column sum's own final
    launch) and sr_vec_fma2_f32: bit-identical to sr_colsum into a scratch row followed by
    sr_vec_fma_f32 per pair (one pair or two)."""
    torch.manual_seed(5)
    big = torch.randn(M, N + 8, device=DEV).to(dtype)
    x = big[:, 4:N + 4]
    m1, m2 = torch.randn(N, device=DEV), torch.randn(N, device=DEV)
    o1, o2 = torch.randn(N, device=DEV), torch.randn(N, device=DEV)
    r1, r2 = o1.clone(), o2.clone()
    tmp = torch.empty(N, device=DEV)
    ops.colsum(x, tmp)
    ops.vec_fma(r1, m1, tmp)
    ops.vec_fma(r2, m2, tmp)
    f1, f2 = o1.clone(), o2.clone()
    ops.colsum_fma(x, [(f1, m1), (f2, m2)])
    g1 = o1.clone()
    ops.colsum_fma(x, [(g1, m1)])
    h1, h2 = o1.clone(), o2.clone()
    ops.vec_fma(h1, m1, tmp, out2=h2, a2=m2)
    torch.cuda.synchronize()
    assert torch.equal(f1, r1) and torch.equal(f2, r2) and torch.equal(g1, r1)
    assert torch.equal(h1, r1) and torch.equal(h2, r2)
    assert rel(r1 - o1, m1 * x.float().sum(0)) < 1e-5


def _ln_ref(x, dy, w, b, eps):
    x = x.detach().clone().requires_grad_(True)
    w = w.detach().clone().requires_grad_(True)
    b = b.detach().clone().requires_grad_(True)
    y = F.layer_norm(x, (x.shape[1],), w, b, eps)
    y.backward(dy)
    return x.grad, w.grad, b.grad


@pytest.mark.parametrize("cols", [384, 1024, 2048])
@pytest.mark.parametrize("dy_dtype", [torch.float32, torch.bfloat16])
def test_layernorm_bwd(ops, cols, dy_dtype):
    torch.manual_seed(5)
    R = 3001
    x = torch.randn(R, cols, device=DEV) * 2 + 0.5
    w = torch.randn(cols, device=DEV)
    b = torch.randn(cols, device=DEV)
    dy = torch.randn(R, cols, device=DEV).to(dy_dtype)
    dx0 = torch.randn(R, cols, device=DEV)
    dx = dx0.clone()
    dxb = torch.empty(R, cols, device=DEV, dtype=torch.bfloat16)
    dw = torch.zeros(cols, device=DEV)
    db = torch.zeros(cols, device=DEV)
    dsum = torch.full((cols,), float("nan"), device=DEV) if cols <= 2048 else None
    ops.layernorm_bwd(x, dy, w, 1e-5, dx, dxb=dxb, dw=dw, db=db, dx_sum=dsum)
    gx, gw, gb = _ln_ref(x, dy.float(), w, b, 1e-5)
    assert rel(dx - dx0, gx) < 1e-5
    assert rel(dxb.float(), dx) < 8e-3
    assert rel(dw, gw) < 1e-5 and rel(db, gb) < 1e-5
    if dsum is not None:  # the fused column sum of the updated rows (proj's bias grad in block_bwd)
        assert rel(dsum, dx.double().sum(0)) < 1e-5


def test_layernorm_bwd_rowmap(ops):
    """Gathered rows (reloc anchor subsample): x rows and dx rows through the map."""
    torch.manual_seed(6)
    R, n, cols = 2000, 300, 1024
    x = torch.randn(R, cols, device=DEV)
    w = torch.randn(cols, device=DEV)
    rowmap = torch.randperm(R, device=DEV)[:n].int()
    dy = torch.randn(n, cols, device=DEV).bfloat16()
    dx = torch.zeros(R, cols, device=DEV)
    dw = torch.zeros(cols, device=DEV)
    db = torch.zeros(cols, device=DEV)
    dsum = torch.empty(cols, device=DEV)
    ops.layernorm_bwd(x, dy, w, 1e-6, dx, rowmap=rowmap, dw=dw, db=db, dx_sum=dsum)
    xs = x[rowmap.long()]
    gx, gw, gb = _ln_ref(xs, dy.float(), w, torch.zeros_like(w), 1e-6)
    ref = torch.zeros_like(dx)
    ref[rowmap.long()] = gx
    assert rel(dx, ref) < 1e-5
    assert rel(dw, gw) < 1e-5 and rel(db, gb) < 1e-5
    assert rel(dsum, dx[rowmap.long()].double().sum(0)) < 1e-5  # over the mapped rows only


def _qk_fwd_ref(raw, C, D, qkv, pos):
    """fp32 statement of the SR_EPI_QKV transform on pre-norm rows (attention.py:72-82)."""
    from oracle.sfm_oracle import rope2d
    M = raw.shape[0]
    H = C // D
    y = raw.view(M, 3, H, D)
    outs = []
    for region, (nw, nb) in enumerate(((qkv["qn_w"], qkv["qn_b"]), (qkv["kn_w"], qkv["kn_b"]))):
        t = F.layer_norm(y[:, region], (D,), nw, nb, qkv["qk_eps"])
        t = rope2d(t.permute(1, 0, 2)[None], pos[None])[0].permute(1, 0, 2)
        outs.append(t)
    outs.append(y[:, 2])
    return torch.stack(outs, 1).reshape(M, 3 * C)


@pytest.mark.parametrize("C,frames,col_offset", [(256, 30, 0), (384, 7, 0), (1024, 4, 1)])
def test_qk_bwd(ops, C, frames, col_offset):
    from sailrecon_amd.layers.rope import RotaryPositionEmbedding2D
    torch.manual_seed(7)
    D, P, gw = 64, 21, 4
    M = frames * P
    raw = (torch.randn(M, 3 * C) * 1.5 + 0.3).bfloat16().float()
    dout = torch.randn(M, 3 * C)
    nrm = [torch.randn(D) for _ in range(4)]
    qkv_cpu = dict(qn_w=nrm[0], qn_b=nrm[1], kn_w=nrm[2], kn_b=nrm[3], qk_eps=1e-5)
    t = torch.arange(M) % P
    p = (t - 5).clamp_min(0)
    pos = torch.stack([p // gw + 1, p % gw + 1], -1) * (t >= 5)[:, None]
    params = [raw] + nrm
    for z in params:
        z.requires_grad_(True)
    _qk_fwd_ref(raw, C, D, dict(qkv_cpu, qn_w=nrm[0], qn_b=nrm[1], kn_w=nrm[2], kn_b=nrm[3]), pos).backward(dout)
    rope = RotaryPositionEmbedding2D(100).tables(D, 5, DEV)
    epi = dict(embed_dim=C, head_dim=D, qk_eps=1e-5, qn_w=nrm[0].detach().to(DEV), qn_b=nrm[1].detach().to(DEV),
               kn_w=nrm[2].detach().to(DEV), kn_b=nrm[3].detach().to(DEV), rope_cos=rope[0], rope_sin=rope[1],
               tokens_per_frame=P, patch_start=5, grid_w=gw, pos_row_base=0)
    lo = C if col_offset else 0
    if col_offset:
        epi["col_offset"] = C
    raw_d = raw.detach()[:, lo:].to(DEV).bfloat16().contiguous()
    d_d = dout[:, lo:].to(DEV).contiguous()
    out = torch.empty(M, 3 * C - lo, device=DEV, dtype=torch.bfloat16)
    grads = torch.zeros(4, D, device=DEV)
    bg0 = torch.randn(3 * C - lo, device=DEV)  # the qkv bias grad, accumulated into
    bg = bg0.clone()
    ops.qk_bwd(raw_d, d_d, out, epi, grads=grads, bias_grad=bg)
    assert rel(out.float().cpu(), raw.grad[:, lo:]) < 8e-3
    assert rel(bg - bg0, out.float().sum(0)) < 1e-5  # column sums of the stored bf16 values
    gref = torch.stack([nrm[0].grad, nrm[1].grad, nrm[2].grad, nrm[3].grad])
    if col_offset:
        assert rel(grads[2:].cpu(), gref[2:]) < 1e-5
    else:
        assert rel(grads.cpu(), gref) < 1e-5


def test_qk_bwd_plain_cast(ops):
    """No qk-norm, no RoPE (DINO blocks): the backward is the bf16 cast of dq|dk|dv."""
    M, C = 500, 384
    d = torch.randn(M, 3 * C, device=DEV)
    out = torch.empty(M, 3 * C, device=DEV, dtype=torch.bfloat16)
    bg = torch.zeros(3 * C, device=DEV)
    ops.qk_bwd(None, d, out, dict(embed_dim=C, head_dim=64), bias_grad=bg)
    assert torch.equal(out, d.bfloat16())
    assert rel(bg, out.float().sum(0)) < 1e-5


def test_cast_nonfinite_adam(ops):
    torch.manual_seed(8)
    src = torch.randn(100, 64, device=DEV)
    dst = torch.empty(100, 64, device=DEV, dtype=torch.bfloat16)
    ops.cast_bf16(src, dst, 0.5)
    assert torch.equal(dst, (src * 0.5).bfloat16())
    n = 10007
    p = torch.randn(n, device=DEV)
    g = torch.randn(n, device=DEV) * 1024.0
    m = torch.zeros(n, device=DEV)
    v = torch.zeros(n, device=DEV)
    scale = torch.tensor([1024.0], device=DEV)
    found = torch.zeros(1, device=DEV, dtype=torch.int32)
    ops.nonfinite_check(g, found, scale)
    assert int(found.item()) == 0
    ref_p = p.clone().requires_grad_(True)
    opt = torch.optim.Adam([ref_p], lr=2e-4, betas=(0.9, 0.999), eps=1e-8)
    for step in (1, 2, 3):
        ref_p.grad = g / 1024.0
        opt.step()
        ops.adam(p, g, m, v, lr=2e-4, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.0, step=step, scale=scale,
                 found_inf=found)
    assert rel(p, ref_p.detach()) < 1e-6
    g[17] = float("inf")
    ops.nonfinite_check(g, found, scale)
    assert int(found.item()) == 1
    p0 = p.clone()
    ops.adam(p, g, m, v, lr=2e-4, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.0, step=4, scale=scale,
             found_inf=found)
    assert torch.equal(p, p0)
    # the 16-B aligned float4 path (with its n % 4 tail) equals the scalar path of misaligned views
    vals = [torch.randn(n, device=DEV) for _ in range(4)]
    vals[3] = vals[3].abs()  # second moments
    al = [t.clone() for t in vals]
    bufs = [torch.empty(n + 1, device=DEV) for _ in range(4)]
    for b, t in zip(bufs, vals):
        b[1:] = t
    mis = [b[1:] for b in bufs]  # 4-B offset: the scalar loop
    for a in (al, mis):
        ops.adam(a[0], a[1], a[2], a[3], lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.01, step=5)
    torch.cuda.synchronize()
    for a, b in zip(al, mis):
        assert torch.equal(a, b)


@pytest.mark.parametrize("mask", [False, True])
def test_attention_bwd_small_f32(ops, mask):
    """Camera-trunk attention backward: fp32, head_dim 128, ~build_lr_mask."""
    torch.manual_seed(9)
    L_, H, D, na = 24, 2, 128, 10
    C = H * D
    qkv = torch.randn(L_, 3 * C, device=DEV)
    g = torch.randn(L_, C, device=DEV)
    d = torch.empty(L_, 3 * C, device=DEV)
    lib = L()
    ops.attention_bwd_small(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], g, d[:, :C], d[:, C:2 * C], d[:, 2 * C:],
                            heads=H, head_dim=D, mask_mode=lib.SR_MASK_CAMERA if mask else lib.SR_MASK_NONE,
                            n_anchor=na)
    q, k, v = (qkv[:, i * C:(i + 1) * C].view(L_, H, D).transpose(0, 1).detach().clone().requires_grad_(True)
               for i in range(3))
    allow = torch.ones(L_, L_, dtype=torch.bool, device=DEV)
    if mask:
        allow = torch.zeros(L_, L_, dtype=torch.bool, device=DEV)
        allow[:, :na] = True
        allow[torch.arange(L_), torch.arange(L_)] = True
    s = (q @ k.transpose(-1, -2)) * D ** -0.5
    o = torch.softmax(s.masked_fill(~allow, float("-inf")), -1) @ v
    o.backward(g.view(L_, H, D).transpose(0, 1))
    for i, t in enumerate((q, k, v)):
        assert rel(d[:, i * C:(i + 1) * C], t.grad.transpose(0, 1).reshape(L_, C)) < 1e-5, "qkv"[i]


def test_fp32_backward_gemms(ops):
    """fp32 dgrad epilogues (F32, GELU_BWD with fp32 aux, split-K BIAS) and the small-row wgrad."""
    torch.manual_seed(10)
    lib = L()
    M, N, K = 24, 256, 768
    a = torch.randn(M, K, device=DEV)
    w = torch.randn(N, K, device=DEV) / 16
    out = torch.empty(M, N, device=DEV)
    ops.gemm(a, w, out, lib.SR_EPI_F32)
    assert rel(out, a @ w.t()) < 1e-5
    ops.gemm(a, w, out, lib.SR_EPI_BIAS)
    assert rel(out, a @ w.t()) < 1e-5
    u = torch.randn(M, N, device=DEV)
    ops.gemm(a, w, out, lib.SR_EPI_GELU_BWD, aux=u)
    gp = 0.5 * (1 + torch.erf(u / math.sqrt(2))) + u * torch.exp(-0.5 * u * u) / math.sqrt(2 * math.pi)
    assert rel(out, (a @ w.t()) * gp) < 1e-5
    dy = torch.randn(M, N, device=DEV)
    dw = torch.randn(N, K, device=DEV)
    dw0 = dw.clone()
    db = torch.zeros(N, device=DEV)
    gam = torch.randn(N, device=DEV)
    wd = torch.randn(N, K, device=DEV)
    rd = torch.zeros(N, device=DEV)
    ops.wgrad_small(dy, a, dw, db=db, accumulate=True, rowscale=gam, wdot=wd, rowdot=rd)
    G = dy.t() @ a
    assert rel(dw, dw0 + gam[:, None] * G) < 1e-5
    assert rel(db, dy.sum(0)) < 1e-5
    assert rel(rd, (wd * G).sum(1)) < 1e-5
    sw = torch.empty(K, N, device=DEV)
    ops.transpose(w, sw, rowscale=gam)
    assert torch.allclose(sw, (w * gam[:, None]).t())


def test_weight_refresh(ops):
    """sr_weight_refresh_bf16 (train/model.py refresh_packs): one launch over a block's four
    weights (ragged 64-row tiles included) gives exactly sr_cast_bf16's forward operand and
    sr_transpose_f32's row-scaled transposed dgrad operand."""
    torch.manual_seed(11)
    shapes = [(3072, 1024), (1024, 1024), (4096, 1000), (1000, 4096)]
    srcs = [torch.randn(r, c, device=DEV) for r, c in shapes]
    scales = [None, torch.randn(1024, device=DEV), None, torch.randn(1000, device=DEV)]
    casts = [torch.empty(r, c, device=DEV, dtype=torch.bfloat16) for r, c in shapes]
    trans = [torch.empty(c, r, device=DEV, dtype=torch.bfloat16) for r, c in shapes]
    ops.weight_refresh(list(zip(srcs, casts, trans, scales)))
    for src, cast, tr, sc in zip(srcs, casts, trans, scales):
        c0 = torch.empty_like(cast)
        t0 = torch.empty_like(tr)
        ops.cast_bf16(src, c0)
        ops.transpose(src, t0, rowscale=sc)
        torch.cuda.synchronize()
        assert torch.equal(cast, c0) and torch.equal(tr, t0)
    # cast-only and transpose-only items
    c1, t1 = torch.empty_like(casts[0]), torch.empty_like(trans[1])
    ops.weight_refresh([(srcs[0], c1, None, None), (srcs[1], None, t1, scales[1])])
    torch.cuda.synchronize()
    assert torch.equal(c1, casts[0]) and torch.equal(t1, trans[1])
    # the whole-model form (sr_weight_refresh_list_bf16): 9 items over a device table, one launch,
    # the same bits per item; re-run after the sources change (the table is reused)
    items = [(src, torch.empty_like(c), torch.empty_like(t), sc) for src, c, t, sc in zip(srcs, casts, trans, scales)]
    items = items + items[:2] + [(srcs[2], torch.empty_like(casts[2]), None, None)] * 2 + \
        [(srcs[3], None, torch.empty_like(trans[3]), scales[3])]
    table = ops.weight_refresh_table(items, DEV)
    for rnd in range(2):
        if rnd:
            for src in srcs:
                src.mul_(-0.5)
        ops.weight_refresh_list(table)
        for src, cast, tr, sc in items:
            if cast is not None:
                c0 = torch.empty_like(cast)
                ops.cast_bf16(src, c0)
                torch.cuda.synchronize()
                assert torch.equal(cast, c0)
            if tr is not None:
                t0 = torch.empty_like(tr)
                ops.transpose(src, t0, rowscale=sc)
                torch.cuda.synchronize()
                assert torch.equal(tr, t0)
