#!/usr/bin/env python
"""Which attention waves of the headline forward run the hand-scheduled sweep, per timer class,
at a given qk-norm gain (bench.py --qk-gain): every bf16 attention launch of one SailRecon.forward
(N=32 @518) gets an sr_attn_desc.sweep_stats counter pair.  The fixed-offset sweep needs each row's
Cauchy-Schwarz bound qb within 2^174 of its score max over the first three key tiles; rows outside
send their wave to the compiled loop.

    python tools/sweep_stats.py [--views 32] [--gains 1,2,3,4]
"""

import argparse
import json
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

    def attention(q, *a, **kw):
        if q.dtype == torch.bfloat16 and kw.get("sweep_stats") is None and kw.get("mask") is None:
            kw["sweep_stats"] = buf(kw.get("tag") or "attn")
        return real_attn(q, *a, **kw)

    def attention_pair(a, b, **kw):
        a, b = dict(a), dict(b)
        a["sweep_stats"] = buf((kw.get("tag") or "pair") + ".a")
        b["sweep_stats"] = buf((kw.get("tag") or "pair") + ".b")
        return real_pair(a, b, **kw)

    ops.attention, ops.attention_pair = attention, attention_pair
    prev = 1.0
    for g in [float(v) for v in args.gains.split(",")]:
        model, _ = bench.build_model(dev)
        bench.scale_qk_gain(model, g)
        stats.clear()
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
            model(images, no_reloc_list=list(range(n)), reloc_list=list(range(n, 2 * n)), fix_rank=300)
        torch.cuda.synchronize()
        print(json.dumps({"qk_gain": g, "waves": {k: {"asm": int(v[0]), "compiled": int(v[1])}
                                                   for k, v in sorted(stats.items())}}), flush=True)
        del model
        torch.cuda.empty_cache()
        prev = g
    del prev


if __name__ == "__main__":
    main()
