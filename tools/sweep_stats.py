#!/usr/bin/env python
"""Which attention waves of the headline forward run the hand-scheduled sweep, per timer class,
at a given qk-norm gain (bench.py --qk-gain): every bf16 attention launch of one SailRecon.forward
(N=32 @518) gets an sr_attn_desc.sweep_stats counter pair.  The fixed-offset sweep needs each row's
upper bound qb within 2^174 of its score max over the first three key tiles; rows outside send
their wave to the compiled loop.  qb is the Cauchy-Schwarz bound c|q| k_bound, or (where that
leaves the window and the key box is on: --box auto) min of it and the per-dimension key box bound
sum_d max(cq_d kmax_d, cq_d kmin_d) (sr_attn_desc.key_box).  --diag also prints, for sampled rows
of the first global launches, the gap of each bound over the row's true score max (log2 units).

    python tools/sweep_stats.py [--views 32] [--gains 1,2,3,4] [--box auto,0] [--diag]
"""

import argparse
import json
import math
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "self-supervise-sfm_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--views", type=int, default=32)
    ap.add_argument("--gains", default="1,2,3,4")
    ap.add_argument("--box", default="auto", help="SR_ATTN_KEY_BOX modes to run, comma-separated")
    ap.add_argument("--diag", action="store_true")
    args = ap.parse_args()
    import bench
    from sailrecon_amd import ops
    dev = torch.device("cuda", 0)
    n = args.views
    x = torch.rand(n, 3, 518, 518, generator=torch.Generator().manual_seed(n))
    images = torch.cat([x, x])[None].to(dev)
    stats = {}

    def buf(tag):
        if tag not in stats:
            stats[tag] = torch.zeros(2, dtype=torch.int32, device=dev)
        return stats[tag]

    real_attn, real_pair = ops.attention, ops.attention_pair
    diag = []

    def gaps(q, k, v, heads, kn, tag):
        """(first 6 launches) quantiles over sampled rows and heads of (bound - true max) for the
        2-norm and box bounds; (every launch) per sampled wave and head the 2-norm bound minus the
        max over the first three key tiles, the value window's upper side per head (sr_attn.hip
        value_window_hi) and the fraction of (wave, head) pairs inside the window"""
        if not args.diag or kn <= 0:
            return
        c = 64 ** -0.5 * 1.4426950408889634
        qt = torch.tensor([0.5, 0.9, 0.99, 1.0], device=q.device)
        f = lambda v: [round(float(x), 1) for x in torch.quantile(torch.cat(v), qt)]  # noqa: E731
        rec = {"tag": tag, "rows": q.shape[0], "keys": k.shape[0]}
        if len(diag) < 6:
            rows = torch.randperm(q.shape[0], generator=torch.Generator().manual_seed(len(diag)))[:64].to(q.device)
            cs, bx = [], []
            for h in range(heads):
                sl = slice(64 * h, 64 * h + 64)
                cq = (q[rows, sl].float() * c)
                kk = k[:, sl].float()
                mx = (cq @ kk.T).max(-1).values
                cs.append(cq.norm(dim=-1) * kn - mx)
                kmax, kmin = kk.max(0).values, kk.min(0).values
                bx.append(torch.maximum(cq * kmax, cq * kmin).sum(-1) - mx)
            rec.update({"cs_gap_q50_90_99_100": f(cs), "box_gap_q50_90_99_100": f(bx)})
        # per wave (64 consecutive query rows): max over its rows of the 2-norm bound minus the
        # row's max over the first three key tiles (the pre-pass the sweep's window is checked on)
        starts = torch.randperm(q.shape[0] // 64, generator=torch.Generator().manual_seed(7))[:16] * 64
        wrows = (starts[:, None] + torch.arange(64)[None]).reshape(-1).to(q.device)
        wv, his, fit = [], [], 0
        lg_l = math.ceil(math.log2(k.shape[0]))
        for h in range(heads):
            sl = slice(64 * h, 64 * h + 64)
            cq = (q[wrows, sl].float() * c)
            mx0 = (cq @ k[:192, sl].float().T).max(-1).values
            w = (cq.norm(dim=-1) * kn * 1.0001 - mx0).view(16, 64).max(-1).values
            vmax = float(v[:, sl].float().abs().max())
            hi = min(max(125 - lg_l - math.ceil(math.log2(max(vmax, 1.0))), 64), 100)
            wv.append(w)
            his.append(hi)
            fit += int((w <= hi + 110).sum())
        rec.update({"wave_cs_gap_mx0_q50_90_99_100": f(wv), "hi_min_max": [min(his), max(his)],
                    "frac_waves_in_window": round(fit / (16 * heads), 3)})
        diag.append(rec)

    def attention(q, *a, **kw):
        if q.dtype == torch.bfloat16 and kw.get("sweep_stats") is None and kw.get("mask") is None:
            kw["sweep_stats"] = buf(kw.get("tag") or "attn")
            if kw.get("tag") == "attn_global":
                gaps(q, a[0], a[1], kw["heads"], kw.get("key_norm_max", 0.0), kw["tag"])
        return real_attn(q, *a, **kw)

    def attention_pair(a, b, **kw):
        a, b = dict(a), dict(b)
        a["sweep_stats"] = buf((kw.get("tag") or "pair") + ".a")
        b["sweep_stats"] = buf((kw.get("tag") or "pair") + ".b")
        gaps(a["q"], a["k0"], a["v0"], kw["heads"], a["key_norm_max"], "pair.a")
        gaps(b["q"], b["k0"], b["v0"], kw["heads"], b["key_norm_max"], "pair.b")
        return real_pair(a, b, **kw)

    ops.attention, ops.attention_pair = attention, attention_pair
    for mode in args.box.split(","):
        ops._KEY_BOX = mode
        for g in [float(v) for v in args.gains.split(",")]:
            model, _ = bench.build_model(dev)
            bench.scale_qk_gain(model, g)
            stats.clear()
            diag.clear()
            with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
                model(images, no_reloc_list=list(range(n)), reloc_list=list(range(n, 2 * n)), fix_rank=300)
            torch.cuda.synchronize()
            print(json.dumps({"qk_gain": g, "key_box": mode,
                              "waves": {k: {"asm": int(v[0]), "compiled": int(v[1])} for k, v in sorted(stats.items())},
                              **({"bound_gaps": diag} if args.diag else {})}), flush=True)
            del model
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
