"""fp8 global attention (BASELINE config 5, "fp8 QKV"; SURVEY §8(d): e4m3 Q/K with per-tensor
scales): sr_quant_fp8 and sr_attention_qk8.

- quantisation: e4m3 (OCP) with one power-of-two exponent e = ceil(log2(amax |mul| / 448)); the
  round trip is checked element-wise against e4m3's 2^-4 relative step.
- attention: the kernel against fp32 softmax attention on the SAME dequantised q8 / k8 (so only the
  bf16 P of the P.V product differs: 1e-2 rel-L2), and against the bf16 kernel on the original q / k
  (the fp8 rounding itself: 5e-2 rel-L2 at these unit-scale inputs).  No reference output pins an
  fp8 contract (the reference runs bf16 SDPA), so the bf16 path remains the default.
"""

import math

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))


def _deq(q8, e):
    return q8.view(torch.float8_e4m3fn).float() * (2.0 ** int(e))


@pytest.mark.parametrize("mul", [1.0, 0.18033688, 37.5])
def test_quant_fp8_roundtrip(mul):
    from sailrecon_amd import ops
    torch.manual_seed(0)
    x = (torch.randn(300, 256, device=DEV) * torch.logspace(-3, 2, 256, device=DEV)).bfloat16()
    q8, e = ops.quant_fp8(x, mul)
    torch.cuda.synchronize()
    ref = x.float() * mul
    amax = float(ref.abs().max())
    e_host = int(e.item())
    assert e_host == math.ceil(math.log2(amax / 448.0)) or amax * 2.0 ** -(e_host - 1) > 448.0
    deq = _deq(q8, e_host)
    assert float(q8.view(torch.float8_e4m3fn).float().abs().max()) <= 448.0
    # e4m3: 3 mantissa bits -> |err| <= 2^-4 |x| for normals, <= 2^-10 * 2^e absolute in the subnormal range
    tol = ref.abs() * 2.0 ** -4 + 2.0 ** (-9 + e_host)
    assert bool(((deq - ref).abs() <= tol).all())


def test_quant_fp8_zero_tensor():
    from sailrecon_amd import ops
    x = torch.zeros(16, 64, device=DEV, dtype=torch.bfloat16)
    q8, e = ops.quant_fp8(x, 1.0)
    torch.cuda.synchronize()
    assert int(e.item()) == 0 and int(q8.float().abs().max()) == 0


@pytest.mark.parametrize("case", ["global", "global_ragged", "frames"])
def test_attention_qk8(case):
    from sailrecon_amd import ops
    torch.manual_seed(1)
    H, D = 4, 64
    C = H * D
    scale = D ** -0.5
    if case == "global":
        B, L = 1, 1024
    elif case == "global_ragged":
        B, L = 1, 700
    else:
        B, L = 3, 150
    x = torch.randn(B * L, 3 * C, device=DEV).bfloat16()
    q, k, v = x[:, :C], x[:, C:2 * C], x[:, 2 * C:]
    kw = dict(batch=B, lq=L, q_bstride=L, l0=L, k0_bstride=L if B > 1 else 0)
    o8 = torch.empty(B * L, C, device=DEV, dtype=torch.bfloat16)
    lse8 = torch.empty(B, H, L, device=DEV)
    ws = ops.Fp8Workspace()
    ops.attention_qk8(q, k, v, o8, heads=H, lse=lse8, ws=ws, **kw)
    o16 = torch.empty_like(o8)
    ops.attention(q, k, v, o16, heads=H, head_dim=D, **kw)
    torch.cuda.synchronize()
    q8, k8, ex = ws.get(B * L, B * L, C, q.device)
    eq, ek = (int(t) for t in ex.tolist()[:2])
    c = scale * math.log2(math.e)
    qd = _deq(q8, eq) / c  # = q as the kernel saw it
    kd = _deq(k8, ek)
    o_ref = torch.empty(B * L, C, device=DEV)
    for b in range(B):
        rs = slice(b * L, (b + 1) * L)
        qh = qd[rs].reshape(L, H, D).transpose(0, 1)
        kh = kd[rs].reshape(L, H, D).transpose(0, 1)
        vh = v[rs].float().reshape(L, H, D).transpose(0, 1)
        s = qh @ kh.transpose(-1, -2) * scale
        o_ref[rs] = (torch.softmax(s, -1) @ vh).transpose(0, 1).reshape(L, C)
        assert torch.allclose(lse8[b], torch.logsumexp(s, -1) / math.log(2), rtol=0, atol=2e-2)
    assert _rel(o8, o_ref) < 1e-2
    assert _rel(o8, o16) < 5e-2


def test_attention_qkv8():
    """q.k^T and P.V in fp8 (global block, one item): against fp32 attention on the dequantised
    q8 / k8 and the e4m3-rounded V (P unrounded: 3e-2 rel-L2 for P's e4m3 rounding), and against
    the bf16 kernel (6e-2)."""
    from sailrecon_amd import ops
    torch.manual_seed(2)
    H, D = 4, 64
    C = H * D
    scale = D ** -0.5
    for L in (1024, 700):
        x = torch.randn(L, 3 * C, device=DEV).bfloat16()
        q, k, v = x[:, :C], x[:, C:2 * C], x[:, 2 * C:]
        kw = dict(batch=1, lq=L, q_bstride=0, l0=L, k0_bstride=0)
        o8 = torch.empty(L, C, device=DEV, dtype=torch.bfloat16)
        ws = ops.Fp8Workspace()
        ops.attention_qk8(q, k, v, o8, heads=H, ws=ws, fp8_v=True, **kw)
        o16 = torch.empty_like(o8)
        ops.attention(q, k, v, o16, heads=H, head_dim=D, **kw)
        torch.cuda.synchronize()
        q8, k8, ex = ws.get(L, L, C, q.device)
        eq, ek, ev = (int(t) for t in ex.tolist())
        amax = float(v.float().abs().max())
        assert ev == math.ceil(math.log2(amax / 448.0)) or amax * 2.0 ** -(ev - 1) > 448.0
        vd = (v.float() * 2.0 ** -ev).to(torch.float8_e4m3fn).float() * 2.0 ** ev
        c = scale * math.log2(math.e)
        qh = (_deq(q8, eq) / c).reshape(L, H, D).transpose(0, 1)
        kh = _deq(k8, ek).reshape(L, H, D).transpose(0, 1)
        vh = vd.reshape(L, H, D).transpose(0, 1)
        o_ref = (torch.softmax(qh @ kh.transpose(-1, -2) * scale, -1) @ vh).transpose(0, 1).reshape(L, C)
        assert _rel(o8, o_ref) < 3e-2, (L, _rel(o8, o_ref))
        assert _rel(o8, o16) < 6e-2, (L, _rel(o8, o16))


def test_aggregator_fp8_global_close_to_bf16():
    """The small aggregator config end to end with the global blocks' q.k^T in fp8 vs bf16."""
    from goldens import rule_state_dict
    from sailrecon_amd.heads.camera_head import CameraHead
    from sailrecon_amd.models.aggregator import Aggregator

    class Hot(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.aggregator = Aggregator(img_size=56, patch_size=14, embed_dim=384, depth=2, num_heads=6,
                                         patch_embed="dinov2_vits14_reg", intermediate_layer_idx=[0, 1])
            self.camera_head = CameraHead(dim_in=768, trunk_depth=2, num_heads=6)

    m = Hot().eval()
    m.load_state_dict(rule_state_dict("small_state_dict_keys.json"))
    m = m.to(DEV)
    x = torch.rand(1, 4, 3, 56, 56, generator=torch.Generator().manual_seed(1)).to(DEV)
    outs = []
    for fp8, fp8_v in ((False, False), (True, False), (True, True)):
        m.aggregator.set_fp8_global(fp8, fp8_v=fp8_v)
        m.aggregator.generator.manual_seed(0)
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
            feats, _, cam = m.aggregator(x, [0, 1], [2, 3], fix_rank=10)
        outs.append((feats[-1].float(), cam.float()))
    m.aggregator.set_fp8_global(False)
    for i in (1, 2):
        assert _rel(outs[i][0], outs[0][0]) < 5e-2
        assert _rel(outs[i][1], outs[0][1]) < 5e-2
