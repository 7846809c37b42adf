"""Op-level parity of every HIP kernel against a plain torch fp32 reference.

All calls go through the C ABI (libsfm_amd.so via sailrecon_amd.ops).
"""

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


def _lib():
    from sailrecon_amd import _lib as L
    return L


DT = [(torch.float32, 2e-6), (torch.bfloat16, 8e-3)]


@pytest.mark.parametrize("dtype,tol", DT)
# M <= 64 and N > 128 take the few-row 64 x 256 tiles (ragged N included)
@pytest.mark.parametrize("M,N,K", [(128, 128, 64), (300, 256, 1024), (1374, 384, 128), (77, 3072, 1024),
                                   (2500, 512, 256), (4100, 1024, 1024), (2048, 256, 4096),
                                   (64, 388, 256), (9, 2052, 128), (40, 200, 64)])
def test_gemm_bias_gelu(ops, dtype, tol, M, N, K):
    L = _lib()
    g = torch.Generator(device="cpu").manual_seed(M + N + K)
    a = torch.randn(M, K, generator=g).to(DEV, dtype)
    w = (torch.randn(N, K, generator=g) / math.sqrt(K)).to(DEV, dtype)
    b = torch.randn(N, generator=g).to(DEV)
    ref = a.float() @ w.float().t() + b
    out = torch.empty(M, N, device=DEV, dtype=dtype)
    ops.gemm(a, w, out, L.SR_EPI_BIAS, bias=b)
    assert rel(out.float(), ref) < tol
    ops.gemm(a, w, out, L.SR_EPI_BIAS_GELU, bias=b)
    assert rel(out.float(), F.gelu(ref)) < tol


@pytest.mark.parametrize("M,N,K", [(8300, 4096, 128), (33000, 1024, 192), (32769, 1024, 64), (87936, 1024, 1024),
                                   (43968, 1024, 4096)])
def test_gemm256_tiles(ops, M, N, K):
    """>= 512 256x256 tiles select the 256x256 bf16 kernel (the production path):
    ragged last M tile (including slabs that start past row M-1), every bf16 epilogue that
    runs on it at this width (the C3 frame / global proj and fc2 shapes included)."""
    L = _lib()
    g = torch.Generator(device="cpu").manual_seed(M + N)
    a = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16)
    w = (torch.randn(N, K, generator=g) / math.sqrt(K)).to(DEV, torch.bfloat16)
    b, gam = torch.randn(N, generator=g).to(DEV), torch.randn(N, generator=g).to(DEV)
    ref = a.float() @ w.float().t() + b
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    ops.gemm(a, w, out, L.SR_EPI_BIAS, bias=b)
    assert rel(out.float(), ref) < 8e-3
    ops.gemm(a, w, out, L.SR_EPI_BIAS_GELU, bias=b)
    assert rel(out.float(), F.gelu(ref)) < 8e-3
    x = torch.randn(M + 64, N, device=DEV)
    x0 = x.clone()
    ops.gemm(a, w, x[32:32 + M], L.SR_EPI_BIAS_RESID, bias=b, gamma=gam)
    assert torch.equal(x[:32], x0[:32]) and torch.equal(x[32 + M:], x0[32 + M:])
    assert rel(x[32:32 + M] - x0[32:32 + M], ref * gam) < 1e-5


@pytest.mark.parametrize("dtype,tol", DT)
@pytest.mark.parametrize("M,N,K,splits", [(64, 2048, 2048, None), (64, 1024, 8192, None), (37, 256, 1024, 4)])
def test_gemm_splitk(ops, dtype, tol, M, N, K, splits):
    """split-K (camera trunk shapes: few rows, long K) for every epilogue it supports."""
    L = _lib()
    g = torch.Generator(device="cpu").manual_seed(M + K)
    a = torch.randn(M, K, generator=g).to(DEV, dtype)
    w = (torch.randn(N, K, generator=g) / math.sqrt(K)).to(DEV, dtype)
    b, gam = torch.randn(N, generator=g).to(DEV), torch.randn(N, generator=g).to(DEV)
    assert (splits or ops._splitk_plan(M, N, K, L.SR_EPI_BIAS, dtype)) > 1
    ref = a.float() @ w.float().t() + b
    out = torch.empty(M, N, device=DEV, dtype=dtype)
    ops.gemm(a, w, out, L.SR_EPI_BIAS, bias=b, splits=splits)
    assert rel(out.float(), ref) < tol
    ops.gemm(a, w, out, L.SR_EPI_BIAS_GELU, bias=b, splits=splits)
    assert rel(out.float(), F.gelu(ref)) < tol
    x = torch.randn(M, N + 8, device=DEV)[:, :N]
    x0 = x.clone()
    ops.gemm(a, w, x, L.SR_EPI_BIAS_RESID, bias=b, gamma=gam, splits=splits)
    assert rel(x - x0, ref * gam) < max(tol, 1e-5)
    o32 = torch.empty(M, N + 4, device=DEV)[:, :N]  # F32: fp32 output for either operand type (dgrad)
    ops.gemm(a, w, o32, L.SR_EPI_F32, bias=b, splits=splits)
    assert rel(o32, ref) < max(tol, 1e-5)


@pytest.mark.parametrize("M,K", [(33000, 1024), (43968, 4096), (8300, 256), (4100, 64)])
def test_gemm_resid_lds_epilogue(ops, M, K):
    """SR_GEMM_RESID_LDS: the 256x256 residual GEMM staging its x tile through LDS by LDS-DMA
    (quarter 0 under the last k-tile, two quarters in flight, whole-row stores) computes exactly
    what the register epilogue computes, in the one-kernel launch, with the 128x128 tail split, and
    in a grouped launch; K = 64 is a single k-tile (quarter 0 into the never-used stage buffer),
    ragged M leaves a partial last row tile on the guarded path."""
    L = _lib()
    g = torch.Generator(device="cpu").manual_seed(M + K)
    N = 1024
    a = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16)
    w = (torch.randn(N, K, generator=g) / math.sqrt(K)).to(DEV, torch.bfloat16)
    b, gam = torch.randn(N, generator=g).to(DEV), torch.randn(N, generator=g).to(DEV)
    x0 = torch.randn(M, N, generator=g).to(DEV)
    outs = []
    for rl in (0, 1):
        for tail in (0, 1):
            x = x0.clone()
            with ops.tuning(SR_GEMM_RESID_LDS=rl, SR_GEMM_TAIL=tail):
                ops.gemm(a, w, x, L.SR_EPI_BIAS_RESID, bias=b, gamma=gam, splits=1)
            outs.append(x)
        x = x0.clone()
        with ops.tuning(SR_GEMM_RESID_LDS=rl):
            h = M // 2
            ops.gemm_group([dict(a=a[:h], w=w, out=x[:h], bias=b, gamma=gam),
                            dict(a=a[h:], w=w, out=x[h:], bias=b, gamma=gam)], L.SR_EPI_BIAS_RESID)
        outs.append(x)
        x = x0.clone()
        with ops.tuning(SR_GEMM_RESID_LDS=rl):  # no bias
            ops.gemm(a, w, x, L.SR_EPI_BIAS_RESID, gamma=gam, splits=1)
        outs.append(x)
    # outs: [register epilogue: one kernel, tail split, grouped, no bias] then the same with RESID_LDS
    for i in (1, 2, 4, 5, 6):
        assert torch.equal(outs[i], outs[0]), i
    assert torch.equal(outs[7], outs[3])
    ref = (a.float() @ w.float().t() + b) * gam
    assert rel(outs[0] - x0, ref) < 1e-5
    assert rel(outs[3] - x0, (a.float() @ w.float().t()) * gam) < 1e-5


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 2e-6), (torch.bfloat16, 1e-5)])
@pytest.mark.parametrize("M", [517, 3000])
def test_gemm_resid_strided(ops, dtype, tol, M):
    """fp32 residual epilogue on a row slice of a bigger buffer (the reloc/global stacks)."""
    L = _lib()
    N, K = 256, 512
    a = torch.randn(M, K, device=DEV).to(dtype)
    w = (torch.randn(N, K, device=DEV) / math.sqrt(K)).to(dtype)
    b, gam = torch.randn(N, device=DEV), torch.randn(N, device=DEV)
    x = torch.randn(M + 100, N, device=DEV)
    x0 = x.clone()
    ops.gemm(a, w, x[50:50 + M], L.SR_EPI_BIAS_RESID, bias=b, gamma=gam)
    ref = x0.clone()
    ref[50:50 + M] += (a.float() @ w.float().t() + b) * gam
    assert torch.equal(x[:50], x0[:50]) and torch.equal(x[50 + M:], x0[50 + M:])
    assert rel(x[50:50 + M] - x0[50:50 + M], ref[50:50 + M] - x0[50:50 + M]) < max(tol, 1e-5)


@pytest.mark.parametrize("dtype,tol", DT)
@pytest.mark.parametrize("frames,npatch,C", [(3, 16, 128), (10, 256, 256)])
def test_gemm_patch_epilogue(ops, dtype, tol, frames, npatch, C):
    L = _lib()
    P, K = npatch + 5, 640
    a = torch.randn(frames * npatch, K, device=DEV).to(dtype)
    w = (torch.randn(C, K, device=DEV) / 25).to(dtype)
    b = torch.randn(C, device=DEV)
    pos = torch.randn(npatch, C, device=DEV)
    x = torch.full((frames * P, C), 7.0, device=DEV)
    w = w / (K ** 0.5 / 25)
    ops.gemm(a, w, x, L.SR_EPI_PATCH, bias=b, rows=frames * npatch,
             patch=dict(seg_rows=npatch, seg_stride=P, seg_offset=5, row_add=pos))
    ref = (a.float() @ w.float().t() + b).view(frames, npatch, C) + pos
    xv = x.view(frames, P, C)
    assert torch.all(xv[:, :5] == 7.0)
    assert rel(xv[:, 5:], ref) < tol


def _rope_ref(t, pos, base=100.0):
    from oracle.sfm_oracle import rope2d
    return rope2d(t, pos, base)


@pytest.mark.parametrize("dtype,tol", DT)
@pytest.mark.parametrize("col_offset", [0, 1])
@pytest.mark.parametrize("frames", [3, 100, 3200])  # 3200 x 21 rows: >= 512 256x256 tiles (bf16 production path)
def test_gemm_qkv_epilogue(ops, dtype, tol, col_offset, frames):
    """bias + qk-LayerNorm + 2-D RoPE fused into the qkv GEMM (attention.py:72-82)."""
    from sailrecon_amd.layers.rope import RotaryPositionEmbedding2D
    L = _lib()
    C, H, D = 256, 4, 64
    P, gw = 21, 4
    M = frames * P
    a = torch.randn(M, C, device=DEV).to(dtype)
    w = (torch.randn(3 * C, C, device=DEV) / 16).to(dtype)
    b = torch.randn(3 * C, device=DEV)
    qn_w, qn_b, kn_w, kn_b = (torch.randn(D, device=DEV) for _ in range(4))
    rope = RotaryPositionEmbedding2D(100).tables(D, 5, DEV)
    wo, bo = (w[C:], b[C:]) if col_offset else (w, b)
    out = torch.empty(M, wo.shape[0], device=DEV, dtype=dtype)
    epi = dict(embed_dim=C, head_dim=D, qk_eps=1e-5, qn_w=qn_w, qn_b=qn_b, kn_w=kn_w, kn_b=kn_b,
               rope_cos=rope[0], rope_sin=rope[1], tokens_per_frame=P, patch_start=5, grid_w=gw, pos_row_base=0,
               col_offset=C if col_offset else 0)
    ops.gemm(a, wo, out, L.SR_EPI_QKV, bias=bo, qkv=epi)
    y = (a.float() @ w.float().t() + b).cpu().view(M, 3, H, D)
    t = torch.arange(M) % P
    p = (t - 5).clamp_min(0)
    pos = torch.stack([p // gw + 1, p % gw + 1], -1) * (t >= 5)[:, None]
    q = F.layer_norm(y[:, 0], (D,), qn_w.cpu(), qn_b.cpu(), 1e-5)
    k = F.layer_norm(y[:, 1], (D,), kn_w.cpu(), kn_b.cpu(), 1e-5)
    q = _rope_ref(q.permute(1, 0, 2)[None], pos[None])[0].permute(1, 0, 2)
    k = _rope_ref(k.permute(1, 0, 2)[None], pos[None])[0].permute(1, 0, 2)
    ref = torch.stack([q, k, y[:, 2]], 1).reshape(M, 3 * C)
    if col_offset:
        ref = ref[:, C:]
    assert rel(out.float().cpu(), ref) < tol


def _attn_ref(q, k, v, scale, mask=None):
    s = (q.double() @ k.double().transpose(-1, -2)) * scale
    if mask is not None:
        s = s.masked_fill(~mask, float("-inf"))
    return (torch.softmax(s, -1) @ v.double()).float()


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 2e-6), (torch.bfloat16, 1e-2)])
@pytest.mark.parametrize("frames,P", [(2, 261), (3, 64), (1, 1374)])
def test_attention_frame(ops, dtype, tol, frames, P):
    H, D = 4, 64
    C = H * D
    qkv = torch.randn(frames * P, 3 * C, device=DEV).to(dtype)
    o = torch.empty(frames * P, C, device=DEV, dtype=dtype)
    ops.attention(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], o, heads=H, head_dim=D, batch=frames, lq=P,
                  q_bstride=P, l0=P, k0_bstride=P)
    t = qkv.float().view(frames, P, 3, H, D).permute(2, 0, 3, 1, 4)
    ref = _attn_ref(t[0], t[1], t[2], D ** -0.5).permute(0, 2, 1, 3).reshape(frames * P, C)
    assert rel(o.float(), ref) < tol


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 2e-6), (torch.bfloat16, 1e-2)])
def test_attention_reloc_segments(ops, dtype, tol):
    """global_reloc: queries see [shared anchor subsample ; own frame] = the reference bool mask."""
    H, D, Nq, P, nsub = 2, 64, 3, 70, 45
    C = H * D
    qkv = torch.randn(Nq * P, 3 * C, device=DEV).to(dtype)
    kv_sub = torch.randn(nsub, 2 * C, device=DEV).to(dtype)
    o = torch.empty(Nq * P, C, device=DEV, dtype=dtype)
    ops.attention(qkv[:, :C], kv_sub[:, :C], kv_sub[:, C:], o, heads=H, head_dim=D, batch=Nq, lq=P, q_bstride=P,
                  l0=nsub, k0_bstride=0, k1=qkv[:, C:2 * C], v1=qkv[:, 2 * C:], l1=P, k1_bstride=P)
    # dense reference over [subsample ; queries] with the reference's allowed set
    # (aggregator.py:302-311, 832-851): anchors see anchors; query frame j sees anchors + frame j
    L_ = nsub + Nq * P
    seq_k = torch.cat([kv_sub[:, :C], qkv[:, C:2 * C]]).float()
    seq_v = torch.cat([kv_sub[:, C:], qkv[:, 2 * C:]]).float()
    seq_q = torch.cat([torch.zeros(nsub, C, device=DEV), qkv[:, :C].float()])
    mask = torch.zeros(L_, L_, dtype=torch.bool)
    mask[:nsub, :nsub] = True
    for j in range(Nq):
        r = slice(nsub + j * P, nsub + (j + 1) * P)
        mask[r, :nsub] = True
        mask[r, r] = True
    mask = mask.to(DEV)
    qh = seq_q.view(L_, H, D).transpose(0, 1)
    kh = seq_k.view(L_, H, D).transpose(0, 1)
    vh = seq_v.view(L_, H, D).transpose(0, 1)
    ref = _attn_ref(qh, kh, vh, D ** -0.5, mask[None]).transpose(0, 1).reshape(L_, C)[nsub:]
    assert rel(o.float(), ref) < tol


@pytest.mark.parametrize("D", [64, 128])
def test_attention_camera_mask_f32(ops, D):
    from sailrecon_amd.heads.camera_head import build_lr_mask
    H, S, na = 3, 11, 6
    C = H * D
    qkv = torch.randn(S, 3 * C, device=DEV)
    o = torch.empty(S, C, device=DEV)
    ops.attention(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], o, heads=H, head_dim=D, batch=1, lq=S, q_bstride=0,
                  l0=S, k0_bstride=0, mask_mode=_lib().SR_MASK_CAMERA, n_anchor=na)
    mask = ~build_lr_mask(S, list(range(na)), device=DEV)[0]
    t = qkv.view(S, 3, H, D).permute(1, 2, 0, 3)
    ref = _attn_ref(t[0], t[1], t[2], D ** -0.5, mask).transpose(0, 1).reshape(S, C)
    assert rel(o, ref) < 2e-6


def test_attention_global_long(ops):
    """one long sequence (global stack shape class), bf16, tail tile ragged."""
    H, D, L_ = 2, 64, 5000
    C = H * D
    qkv = torch.randn(L_, 3 * C, device=DEV).bfloat16()
    o = torch.empty(L_, C, device=DEV, dtype=torch.bfloat16)
    ops.attention(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], o, heads=H, head_dim=D, batch=1, lq=L_, q_bstride=0,
                  l0=L_, k0_bstride=0)
    t = qkv.float().view(L_, 3, H, D).permute(1, 2, 0, 3)
    ref = _attn_ref(t[0], t[1], t[2], D ** -0.5).transpose(0, 1).reshape(L_, C)
    assert rel(o.float(), ref) < 1e-2


@pytest.mark.parametrize("case", ["frame", "global", "reloc"])
def test_attention_wide_tiles(ops, case):
    """shapes with >= 512 256-row workgroups select the production 256-row tiles (the small
    tests above run the 128-row fallback); bf16, ragged tails."""
    H, D = 16, 64
    C = H * D
    if case == "frame":
        B, P = 64, 261
        qkv = torch.randn(B * P, 3 * C, device=DEV).bfloat16()
        o = torch.empty(B * P, C, device=DEV, dtype=torch.bfloat16)
        ops.attention(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], o, heads=H, head_dim=D, batch=B, lq=P,
                      q_bstride=P, l0=P, k0_bstride=P)
        t = qkv.float().view(B, P, 3, H, D).permute(2, 0, 3, 1, 4)
        ref = _attn_ref(t[0], t[1], t[2], D ** -0.5).permute(0, 2, 1, 3).reshape(B * P, C)
    elif case == "global":
        L_ = 8100
        qkv = torch.randn(L_, 3 * C, device=DEV).bfloat16()
        o = torch.empty(L_, C, device=DEV, dtype=torch.bfloat16)
        ops.attention(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], o, heads=H, head_dim=D, batch=1, lq=L_,
                      q_bstride=0, l0=L_, k0_bstride=0)
        t = qkv.float().view(L_, 3, H, D).permute(1, 2, 0, 3)
        ref = torch.cat([_attn_ref(t[0][h:h + 1], t[1][h:h + 1], t[2][h:h + 1], D ** -0.5) for h in range(H)])
        ref = ref.transpose(0, 1).reshape(L_, C)
    else:
        Nq, P, nsub = 64, 130, 300
        qkv = torch.randn(Nq * P, 3 * C, device=DEV).bfloat16()
        kv = torch.randn(nsub, 2 * C, device=DEV).bfloat16()
        o = torch.empty(Nq * P, C, device=DEV, dtype=torch.bfloat16)
        ops.attention(qkv[:, :C], kv[:, :C], kv[:, C:], o, heads=H, head_dim=D, batch=Nq, lq=P, q_bstride=P,
                      l0=nsub, k0_bstride=0, k1=qkv[:, C:2 * C], v1=qkv[:, 2 * C:], l1=P, k1_bstride=P)
        t = qkv.float().view(Nq, P, 3, H, D).permute(2, 0, 3, 1, 4)        # [3, Nq, H, P, D]
        ks = kv[:, :C].float().view(nsub, H, D).transpose(0, 1)[None].expand(Nq, H, nsub, D)
        vs = kv[:, C:].float().view(nsub, H, D).transpose(0, 1)[None].expand(Nq, H, nsub, D)
        ref = _attn_ref(t[0], torch.cat([ks, t[1]], 2), torch.cat([vs, t[2]], 2), D ** -0.5)
        ref = ref.permute(0, 2, 1, 3).reshape(Nq * P, C)
    assert rel(o.float(), ref) < 1e-2


def test_attention_softmax_spike(ops):
    """force the online-softmax rescale branch late in the key sweep (rule 26)."""
    H, D, L_ = 1, 64, 700
    C = H * D
    qkv = torch.randn(L_, 3 * C, device=DEV) * 0.1
    qkv[:, :C] = 1.0
    qkv[650, C:2 * C] = 3.0  # one key row scores far above the rest
    for dt, tol in ((torch.float32, 2e-6), (torch.bfloat16, 1e-2)):
        x = qkv.to(dt)
        o = torch.empty(L_, C, device=DEV, dtype=dt)
        ops.attention(x[:, :C], x[:, C:2 * C], x[:, 2 * C:], o, heads=H, head_dim=D, batch=1, lq=L_, q_bstride=0,
                      l0=L_, k0_bstride=0)
        t = x.float().view(L_, 3, H, D).permute(1, 2, 0, 3)
        ref = _attn_ref(t[0], t[1], t[2], D ** -0.5).transpose(0, 1).reshape(L_, C)
        assert rel(o.float(), ref) < tol


@pytest.mark.parametrize("cols", [384, 1024, 4096])
def test_layernorm_copy(ops, cols):
    """sr_layernorm_copy (the training tape's x0 / x1 in the LayerNorm pass): the normalised rows
    bit-identical to sr_layernorm's and the copy equal to the input rows, at a padded row stride."""
    torch.manual_seed(cols)
    R = 1377
    x = torch.randn(R, cols, device=DEV) * 3 + 1
    w, b = torch.randn(cols, device=DEV), torch.randn(cols, device=DEV)
    o0 = torch.empty(R, cols, device=DEV, dtype=torch.bfloat16)
    o1 = torch.empty_like(o0)
    xc = torch.full((R, cols + 64), float("nan"), device=DEV)[:, :cols]
    ops.layernorm(x, w, b, 1e-6, o0)
    ops.layernorm(x, w, b, 1e-6, o1, x_copy=xc)
    torch.cuda.synchronize()
    assert torch.equal(o0, o1) and torch.equal(xc, x)


@pytest.mark.parametrize("cols", [384, 768, 1024, 2048])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_layernorm_rowmap(ops, cols, dtype):
    x = torch.randn(300, cols, device=DEV) * 3 + 1
    w, b = torch.randn(cols, device=DEV), torch.randn(cols, device=DEV)
    rm = torch.randint(0, 300, (123,), device=DEV, dtype=torch.int32)
    out = torch.empty(123, cols, device=DEV, dtype=dtype)
    ops.layernorm(x, w, b, 1e-5, out, rowmap=rm)
    ref = F.layer_norm(x[rm.long()], (cols,), w, b, 1e-5)
    assert rel(out.float(), ref) < (1e-6 if dtype == torch.float32 else 5e-3)
    out2 = torch.empty(300, cols, device=DEV)
    ops.layernorm(x, None, None, 1e-6, out2)
    assert rel(out2, F.layer_norm(x, (cols,), eps=1e-6)) < 1e-6


@pytest.mark.parametrize("cols", [256, 768, 1024, 2048])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_residual_layernorm(ops, cols, dtype):
    """x += gamma * y (y strided inside a wider buffer, as the projection output in the qkv slot),
    out = LN(x): x exact against the fp32 update, out against F.layer_norm; gamma None = 1; ragged
    row counts (the 4-rows-per-wave tail)."""
    for rows in (1, 7, 301):
        x = torch.randn(rows, cols, device=DEV) * 3 + 1
        ybuf = torch.randn(rows, 3 * cols, device=DEV).to(dtype)
        y = ybuf[:, cols:2 * cols]
        g, w, b = (torch.randn(cols, device=DEV) for _ in range(3))
        for gamma in (g, None):
            x0 = x.clone()
            out = torch.empty(rows, cols, device=DEV, dtype=dtype)
            ops.residual_layernorm(x, y, gamma, w, b, 1e-6, out)
            xr = x0 + y.float() * (gamma if gamma is not None else 1.0)
            assert rel(x, xr) < 1e-6
            ref = F.layer_norm(xr, (cols,), w, b, 1e-6)
            assert rel(out.float(), ref) < (1e-6 if dtype == torch.float32 else 5e-3)
            x = x0
    with pytest.raises(ValueError):
        ops.residual_layernorm(x, torch.empty(rows, 320, device=DEV, dtype=dtype), None, w, b, 1e-6, out)


def test_im2col_and_tokens(ops):
    img = torch.rand(2, 3, 28, 42, device=DEV)
    out = torch.empty(2 * 6, 640, device=DEV)
    ops.im2col_normalize(img, 14, out, 640)
    mean = torch.tensor([0.485, 0.456, 0.406], device=DEV).view(1, 3, 1, 1)
    std = torch.tensor([0.229, 0.224, 0.225], device=DEV).view(1, 3, 1, 1)
    ref = F.unfold((img - mean) / std, 14, stride=14).transpose(1, 2).reshape(12, 588)
    assert rel(out[:, :588], ref) < 1e-6 and torch.all(out[:, 588:] == 0)
    x = torch.zeros(4 * 10, 8, device=DEV)
    table = torch.randn(3, 2, 8, device=DEV)
    types = torch.tensor([0, 1, 2, 1], dtype=torch.int32, device=DEV)
    ops.set_special_tokens(x, 4, 10, table, types)
    xv = x.view(4, 10, 8)
    for f, t in enumerate([0, 1, 2, 1]):
        assert torch.equal(xv[f, :2], table[t]) and torch.all(xv[f, 2:] == 0)


def test_small_fp32_ops(ops):
    a = torch.randn(7, 9, device=DEV)
    w, b = torch.randn(33, 9, device=DEV), torch.randn(33, device=DEV)
    out = torch.empty(7, 33, device=DEV)
    ops.linear_small(a, w, b, out, rows=7)
    assert rel(out, a @ w.t() + b) < 1e-6
    ops.linear_small(a, w, b, out, rows=7, act_in=1)
    assert rel(out, F.silu(a) @ w.t() + b) < 1e-6
    a2 = torch.randn(5, 1024, device=DEV)
    w2, b2 = torch.randn(9, 1024, device=DEV), torch.randn(9, device=DEV)
    o2 = torch.empty(5, 9, device=DEV)
    ops.linear_small(a2, w2, b2, o2, rows=5)
    assert rel(o2, a2 @ w2.t() + b2) < 1e-6
    y = torch.empty_like(a2)
    ops.silu(a2, y)
    assert rel(y, F.silu(a2)) < 1e-6
    xn, x0, mod = torch.randn(5, 64, device=DEV), torch.randn(5, 64, device=DEV), torch.randn(5, 192, device=DEV)
    o3 = torch.empty(5, 64, device=DEV)
    ops.adaln_modulate(xn, x0, mod, o3)
    sh, scl, gt = mod.chunk(3, -1)
    assert rel(o3, gt * (xn * (1 + scl) + sh) + x0) < 1e-6
    pred, delta, act = torch.zeros(5, 9, device=DEV), torch.randn(5, 9, device=DEV), torch.empty(5, 9, device=DEV)
    ops.pose_update(pred, delta, act, first=True)
    ops.pose_update(pred, delta, act, first=False)
    assert torch.allclose(pred, 2 * delta)
    assert torch.allclose(act, torch.cat([2 * delta[:, :7], F.relu(2 * delta[:, 7:])], -1))
    from oracle.sfm_oracle import pose_encoding_to_extri_intri
    enc = torch.randn(1, 5, 9)
    enc[..., 7:] = enc[..., 7:].abs() + 0.3
    ext, intr = torch.empty(5, 3, 4, device=DEV), torch.empty(5, 3, 3, device=DEV)
    ops.pose_decode(enc[0].to(DEV), (224, 300), ext, intr)
    re, ri = pose_encoding_to_extri_intri(enc, (224, 300))
    assert rel(ext.cpu(), re[0]) < 1e-6 and rel(intr.cpu(), ri[0]) < 1e-6


@pytest.mark.parametrize("epi_name", ["QKV", "BIAS", "BIAS_RESID", "BIAS_GELU_AUX", "QKV_AUX"])
def test_gemm_group(ops, epi_name):
    """sr_gemm_group: 3 independent bf16 GEMMs of one epilogue in ONE 256x256 launch (different M
    and N, one problem's workgroup count not a multiple of 8) are bit-identical to the same
    problems launched apart on the 256x256 kernel (>= 512 tiles each) -- and, QKV, the layer's
    query / anchor / subsample-K|V projections with the qk-LayerNorm + RoPE epilogue.  *_AUX: with
    the training forward's saved pre-activation / pre-norm q|k|v output (aux), as
    train.engine.run_block_train_multi groups the layer's reloc and global blocks."""
    from sailrecon_amd.layers.rope import RotaryPositionEmbedding2D
    L = _lib()
    with_aux = epi_name.endswith("_AUX")
    epi_name = epi_name[:-4] if with_aux else epi_name
    epi = getattr(L, "SR_EPI_" + epi_name)
    C, H, D, P, gw = 1024, 16, 64, 21, 4
    g = torch.Generator(device=DEV).manual_seed(3)
    rope = RotaryPositionEmbedding2D(100).tables(D, 5, DEV)
    probs, plain = [], []
    # (rows, N): 2,064 / 516 / 552 tiles of 256x256, all >= 512 (the 256x256 kernel when apart); 516 is
    # not a multiple of 8 (4 padding workgroups); ragged last row tiles in the second and third
    for i, (M, N) in enumerate(((172 * 256, 3072), (43 * 256 - 100, 3072), (69 * 256 - 5, 2048))):
        a = torch.randn(M, C, device=DEV, generator=g).bfloat16()
        w = (torch.randn(3 * C, C, device=DEV, generator=g) / 32).bfloat16()[3 * C - N:]
        b = torch.randn(N, device=DEV, generator=g)
        gm = torch.randn(N, device=DEV, generator=g)
        p = dict(a=a, w=w, bias=b)
        if epi_name == "QKV":
            qn = [torch.randn(D, device=DEV, generator=g) for _ in range(4)]
            p["qkv"] = dict(embed_dim=C, head_dim=D, qk_eps=1e-5, qn_w=qn[0], qn_b=qn[1], kn_w=qn[2], kn_b=qn[3],
                            rope_cos=rope[0], rope_sin=rope[1], tokens_per_frame=P, patch_start=5, grid_w=gw,
                            pos_row_base=7 * i, col_offset=3 * C - N)
        if epi_name == "BIAS_RESID":
            p["gamma"] = gm
            x0 = torch.randn(M, N, device=DEV, generator=g)
            p["out"], ref_out = x0.clone(), x0.clone()
        else:
            p["out"] = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
            ref_out = torch.empty_like(p["out"])
        if with_aux:
            p["aux"] = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
            p["ref_aux"] = torch.empty_like(p["aux"])
        probs.append(p)
        plain.append(ref_out)
    ops.gemm_group(probs, epi)
    with ops.tuning(SR_GEMM_TAIL=0):  # sr_gemm on the 256x256 kernel alone (no 128x128 tail launch)
        for p, ref_out in zip(probs, plain):
            ops.gemm(p["a"], p["w"], ref_out, epi, bias=p["bias"], gamma=p.get("gamma"), qkv=p.get("qkv"),
                     aux=p.get("ref_aux"), splits=1)
    torch.cuda.synchronize()
    for p, ref_out in zip(probs, plain):
        assert torch.equal(p["out"], ref_out)
        if with_aux:
            assert torch.equal(p["aux"], p["ref_aux"])


@pytest.mark.parametrize("epi_name", ["F32", "GELU_BWD"])
def test_gemm_group_dgrad(ops, epi_name):
    """sr_gemm_group with the training dgrads' epilogues (F32: fp32 out; GELU_BWD: dU = GELU'(u) *
    (a . w) with the saved pre-activation u as aux), as train.engine.block_bwd_multi groups the
    layer's reloc and global blocks: bit-identical to the problems launched apart on the 256x256
    kernel (>= 512 tiles each)."""
    L = _lib()
    epi = getattr(L, "SR_EPI_" + epi_name)
    g = torch.Generator(device=DEV).manual_seed(5)
    probs, plain = [], []
    for M, N, K in ((43 * 256 - 100, 4096, 1024), (86 * 256 - 32, 2048, 4096)) if epi_name == "F32" else \
            ((43 * 256 - 100, 4096, 1024), (40 * 256, 4096, 1024)):
        a = torch.randn(M, K, device=DEV, generator=g).bfloat16()
        w = (torch.randn(N, K, device=DEV, generator=g) / 32).bfloat16()
        p = dict(a=a, w=w)
        if epi_name == "GELU_BWD":
            p["aux"] = torch.randn(M, N, device=DEV, generator=g).bfloat16()
            p["out"] = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        else:
            p["out"] = torch.empty(M, N, device=DEV)
        probs.append(p)
        plain.append(torch.empty_like(p["out"]))
    ops.gemm_group(probs, epi)
    with ops.tuning(SR_GEMM_TAIL=0):
        for p, ref_out in zip(probs, plain):
            ops.gemm(p["a"], p["w"], ref_out, epi, aux=p.get("aux"), splits=1)
    torch.cuda.synchronize()
    for p, ref_out in zip(probs, plain):
        assert torch.isfinite(p["out"].float()).all()
        assert torch.equal(p["out"], ref_out)


@pytest.mark.parametrize("var", range(8))
def test_residual_layernorm_variants(ops, var):
    """Every sr_residual_layernorm variant of the SR_RLN_WIDE switch (16-B lanes, two rows per
    wave, non-temporal x stores) computes the same update and LayerNorm: x bit-identical to the
    default variant's (one fused multiply-add per element in every layout) and within fp32
    rounding of x + g*y in fp64; out within bf16 rounding of the reference."""
    rows, cols = 301, 1024
    gen = torch.Generator(device=DEV).manual_seed(5)
    x0 = torch.randn(rows, cols, device=DEV, generator=gen) * 3 + 1
    y = torch.randn(rows, cols, device=DEV, generator=gen).bfloat16()
    g, w, b = (torch.randn(cols, device=DEV, generator=gen) for _ in range(3))
    xr = (x0.double() + y.double() * g.double())
    xd, outd = x0.clone(), torch.empty(rows, cols, device=DEV, dtype=torch.bfloat16)
    x, out = x0.clone(), torch.empty_like(outd)
    with ops.tuning(SR_RLN_WIDE=0):
        ops.residual_layernorm(xd, y, g, w, b, 1e-6, outd)
    with ops.tuning(SR_RLN_WIDE=var):
        ops.residual_layernorm(x, y, g, w, b, 1e-6, out)
    torch.cuda.synchronize()
    assert torch.equal(x, xd)
    assert rel(x, xr) < 1e-7
    assert rel(out.float(), F.layer_norm(xr.float(), (cols,), w, b, 1e-6)) < 5e-3


@pytest.mark.parametrize("rows,n_inst,heads,ld", [(1, 1, 1, 64), (1374, 1, 16, 3072), (305, 7, 16, 1024),
                                                  (777, 3, 24, 1600), (4099, 2, 32, 2048), (64, 300, 8, 512)])
def test_attention_key_box(ops, rows, n_inst, heads, ld):
    """sr_attention_key_box: per (instance, head, dim) max / min of bf16 keys, bit-exact against
    torch amax / amin, with signed zeros, infinities and ragged row counts; instances inst_stride
    rows apart (here rows + 5) inside a wider row stride; scratch pre-filled with NaN (every
    partial slot the reduction reads is written first)."""
    stride = rows + 5
    g = torch.Generator(device=DEV).manual_seed(rows + heads)
    buf = (torch.randn(n_inst * stride, ld, device=DEV, generator=g) * 3).bfloat16()
    buf[0, 0] = -0.0
    buf[min(1, rows - 1), 1] = float("inf")
    buf[0, 2] = float("-inf")
    out = torch.empty(n_inst, heads, 2, 64, device=DEV)
    n2 = torch.full((n_inst, heads), -1.0, device=DEV)
    L = _lib().load()
    sc = torch.full((L.sr_attention_key_box_scratch(rows, n_inst, heads),), float("nan"), device=DEV)
    rc = L.sr_attention_key_box(ops._stream(buf), buf.data_ptr(), ld, rows, stride, n_inst, heads, out.data_ptr(),
                                n2.data_ptr(), sc.data_ptr())
    assert rc == 0
    k = buf.float().view(n_inst, stride, ld)[:, :rows, :heads * 64].reshape(n_inst, rows, heads, 64)
    assert torch.equal(out[:, :, 0], k.amax(1)) and torch.equal(out[:, :, 1], k.amin(1))
    # max |k|^2 per instance and head (fp32 sums: summation order differs from torch's)
    ref = k.double().square().sum(-1).amax(1)
    fin = torch.isfinite(ref)
    assert torch.equal(torch.isinf(n2), ~fin)
    assert torch.allclose(n2[fin].double(), ref[fin], rtol=1e-6, atol=0)


@pytest.mark.parametrize("epi_name", ["BIAS", "BIAS_GELU", "BIAS_RESID", "QKV", "F32", "GELU_BWD",
                                      "BIAS_GELU_AUX", "QKV_ROWMAP_AUX", "QKV_QSCALE", "BIAS_QSCALE"])
@pytest.mark.parametrize("M,N", [(43 * 256 - 100, 3072), (87936, 1024), (2 * 5496, 4096)])
def test_gemm_tail_split(ops, epi_name, M, N):
    """SR_GEMM_TAIL: the rows past the 256x256 kernel's last whole workgroup round run on the
    128x128 kernel in a second launch (frame-sharded ranks' and C3's QKV / proj / fc2 sizes: 516
    tiles = 2 rounds + 4; 1,376 = 5 + 96; 688 = 2 + 176).  Same function as the one-kernel launch:
    within 1e-6 rel (fp32 accumulation in the same k order; the epilogues may contract differently);
    the time-dominant kernel is still reported."""
    from sailrecon_amd.layers.rope import RotaryPositionEmbedding2D
    L = _lib()
    base = {"BIAS_GELU_AUX": "BIAS_GELU", "QKV_ROWMAP_AUX": "QKV", "QKV_QSCALE": "QKV",
            "BIAS_QSCALE": "BIAS"}.get(epi_name, epi_name)
    epi = getattr(L, "SR_EPI_" + base)
    K, C = 1024, 1024
    g = torch.Generator(device=DEV).manual_seed(M + N)
    a = torch.randn(M, K, device=DEV, generator=g).bfloat16()
    w = (torch.randn(N, K, device=DEV, generator=g) / 32).bfloat16()
    kw = dict(bias=torch.randn(N, device=DEV, generator=g))
    aux1 = aux0 = None
    if base == "QKV":
        if N % C:
            pytest.skip("QKV needs whole q|k|v blocks")
        rope = RotaryPositionEmbedding2D(100).tables(64, 40, DEV)
        qn = [torch.randn(64, device=DEV, generator=g) for _ in range(4)]
        kw["qkv"] = dict(embed_dim=C, head_dim=64, qk_eps=1e-5, qn_w=qn[0], qn_b=qn[1], kn_w=qn[2], kn_b=qn[3],
                         rope_cos=rope[0], rope_sin=rope[1], tokens_per_frame=1374, patch_start=5, grid_w=37,
                         pos_row_base=11, col_offset=3 * C - N)
        if epi_name == "QKV_ROWMAP_AUX":  # the anchor-subsample form: positions through a row map
            kw["qkv"].pop("pos_row_base")
            kw["qkv"]["pos_rowmap"] = torch.randint(0, 64 * 1374, (M,), device=DEV, dtype=torch.int32,
                                                    generator=g)
    if epi_name in ("QKV_QSCALE", "BIAS_QSCALE"):
        if base == "QKV" and N != 3 * C:
            pytest.skip("the Q block needs a full q|k|v output")
        kw["q_scale"], kw["q_cols"] = 0.125 * 1.4426950408889634, C
    if epi_name in ("BIAS_GELU_AUX", "QKV_ROWMAP_AUX"):
        aux1 = torch.zeros(M, N, device=DEV, dtype=torch.bfloat16)
        aux0 = torch.zeros_like(aux1)
    if epi_name == "BIAS_RESID":
        kw["gamma"] = torch.randn(N, device=DEV, generator=g)
    if epi_name == "GELU_BWD":
        kw = dict(aux=torch.randn(M, N, device=DEV, generator=g).bfloat16())
    if epi_name in ("BIAS_RESID", "F32"):
        x0 = torch.randn(M, N, device=DEV, generator=g)
        out1, out0 = x0.clone(), x0.clone()
    else:
        out1 = torch.zeros(M, N, device=DEV, dtype=torch.bfloat16)
        out0 = torch.zeros_like(out1)
    kw1, kw0 = dict(kw), dict(kw)
    if aux1 is not None:
        kw1["aux"], kw0["aux"] = aux1, aux0
    with ops.tuning(SR_GEMM_TAIL=1):
        ops.gemm(a, w, out1, epi, splits=1, **kw1)
        k1 = ops.last_kernel()
    with ops.tuning(SR_GEMM_TAIL=0):
        ops.gemm(a, w, out0, epi, splits=1, **kw0)
        k0 = ops.last_kernel()
    torch.cuda.synchronize()
    assert k1 == k0 and k0.startswith("gemm256_kernel"), (k1, k0)
    same = torch.equal(out1, out0)
    print(f"{epi_name} M={M} N={N}: bit-identical={same} rel={rel(out1.float(), out0.float()):.2e}")
    assert rel(out1.float(), out0.float()) < 1e-6
    if aux1 is not None:  # the saved pre-activation rows of the tail launch land in the right rows
        assert rel(aux1.float(), aux0.float()) < 1e-6 and aux1.abs().sum() > 0
    if "QSCALE" in epi_name:  # only the Q block is scaled, before the one rounding
        kw.pop("q_scale"), kw.pop("q_cols")
        plain = torch.zeros_like(out1)
        ops.gemm(a, w, plain, epi, splits=1, **kw)
        torch.cuda.synchronize()
        c = 0.125 * 1.4426950408889634
        assert torch.equal(out1[:, C:], plain[:, C:])
        assert rel(out1[:, :C].float(), plain[:, :C].float() * c) < 4e-3


def test_merge_with_empty_partial(ops):
    """a merge partial with LSE = -inf (no key of that part attended) contributes
    nothing -- in the attention's merge-in epilogue (sr_attn_desc.merge_o) and in sr_attn_merge_n
    alike (mx == -inf guard): the result is the other part's, finite, not NaN."""
    H, D, lq, L = 4, 64, 300, 256
    C = H * D
    g = torch.Generator(device=DEV).manual_seed(31)
    q, k, v = (torch.randn(n, C, device=DEV, generator=g).bfloat16() for n in (lq, L, L))
    o_ref = torch.empty(lq, C, device=DEV, dtype=torch.bfloat16)
    lse_ref = torch.empty(H, lq, device=DEV)
    ops.attention(q, k, v, o_ref, heads=H, head_dim=D, batch=1, lq=lq, q_bstride=0, l0=L, k0_bstride=0, lse=lse_ref)
    junk = torch.randn(lq, C, device=DEV, generator=g).bfloat16()
    empty = torch.full((H, lq), float("-inf"), device=DEV)
    # merge-in epilogue: every row's other part is empty
    o = torch.empty_like(o_ref)
    ops.attention(q, k, v, o, heads=H, head_dim=D, batch=1, lq=lq, q_bstride=0, l0=L, k0_bstride=0,
                  merge_o=junk, merge_lse=empty)
    # N-way merge: part 1 empty
    parts = torch.cat([o_ref, junk])
    lse_parts = torch.stack([lse_ref, empty]).contiguous()
    out = torch.empty_like(o_ref)
    lse_out = torch.empty(H, lq, device=DEV)
    ops.attn_merge_n(parts, lse_parts, out, parts=2, rows=lq, heads=H, head_dim=D, lse_out=lse_out)
    torch.cuda.synchronize()
    for t in (o, out):
        assert torch.isfinite(t.float()).all()
        assert rel(t.float(), o_ref.float()) < 1e-2
    assert torch.equal(out, o_ref) and torch.equal(lse_out, lse_ref)


@pytest.mark.parametrize("M,N,K", [(43968, 4096, 1024), (43 * 256 - 100, 3072, 1024), (300, 256, 128)])
def test_gemm_gelu_bwd_colsum(ops, M, N, K):
    """sr_gemm_epi.colsum (ABI 1.4): the GELU_BWD epilogue's per-64-row-block column sums of its bf16
    output dH -- the 256x256 kernel with and without the tail split, the 128x128 kernel and a grouped
    launch -- equal the column sums of the stored dH to fp32 summation order, and the output itself
    is unchanged."""
    L = _lib()
    g = torch.Generator(device=DEV).manual_seed(M + N)
    a = torch.randn(M, K, device=DEV, generator=g).bfloat16()
    w = (torch.randn(N, K, device=DEV, generator=g) / 32).bfloat16()
    u = torch.randn(M, N, device=DEV, generator=g).bfloat16()
    nb = ops.colsum_blocks(M)
    ref_out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    ops.gemm(a, w, ref_out, L.SR_EPI_GELU_BWD, aux=u)
    torch.cuda.synchronize()
    ref = ref_out.float().sum(0)
    runs = []
    for tail in (0, 1):
        out = torch.empty_like(ref_out)
        cs = torch.full((nb, N), float("nan"), device=DEV)
        with ops.tuning(SR_GEMM_TAIL=tail):
            ops.gemm(a, w, out, L.SR_EPI_GELU_BWD, aux=u, colsum=cs)
        runs.append((out, cs))
    if N % 256 == 0:
        out = torch.empty_like(ref_out)
        cs = torch.full((nb, N), float("nan"), device=DEV)
        h = (M // 2) // 64 * 64
        ops.gemm_group([dict(a=a[:h], w=w, out=out[:h], aux=u[:h], colsum=cs[:h // 64]),
                        dict(a=a[h:], w=w, out=out[h:], aux=u[h:], colsum=cs[h // 64:])], L.SR_EPI_GELU_BWD)
        runs.append((out, cs))
    torch.cuda.synchronize()
    for out, cs in runs:
        assert torch.equal(out, ref_out)
        assert torch.isfinite(cs).all()
        assert rel(cs.sum(0), ref) < 1e-5
        assert rel(cs[-1], ref_out[(nb - 1) * 64:].float().sum(0)) < 1e-5  # the last, ragged block
