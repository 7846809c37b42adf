#!/usr/bin/env python
"""Per-rank rehearsal of the frame-sharded forward on ONE GPU: rank r of a
G-rank SailRecon.forward at N views @518 (bf16 aggregator, fp32 camera head), with the K/V
all-gathers replaced by buffers that keep their contents (aggregator.RankSim).  The rank computes
exactly its share of the real run, so its step time is what each GPU of the driver's G-GPU run
should spend on compute; the gathers (22.5 MB per rank shard per global layer at C3, ~0.15 ms over
xGMI) and their overlap are the part this does not measure.

    python tools/rank_sim.py [--views 32] [--worlds 1,2,4,8] [--rank 0] [--steps 5]

Prints one JSON line per G: step ms (HIP events around the steps), host submit ms (the Python /
C-ABI launch sequence of one step started on an idle GPU: the time the host needs to stay ahead),
and the per-class kernel time split.  Environment switches (SR_RELOC_SPLIT_MIN_WG, SR_SHARD_TAIL,
SR_GROUP_TAILS ...) apply as in the model.  Outputs are not the model's (peers' K/V are stale).
"""

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "self-supervise-sfm_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--views", type=int, default=32)
    ap.add_argument("--img", type=int, default=518)
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    args = ap.parse_args()
    from bench import build_model
    from sailrecon_amd import ops
    from sailrecon_amd.models.aggregator import RankSim, shard_range

    dev = torch.device("cuda", 0)
    model, _ = build_model(dev)
    n = args.views
    x = torch.rand(n, 3, args.img, args.img, generator=torch.Generator().manual_seed(n))
    images = torch.cat([x, x])[None].to(dev)
    no_reloc, reloc = list(range(n)), list(range(n, 2 * n))

    def step():
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
            return model(images, no_reloc_list=no_reloc, reloc_list=reloc, fix_rank=300)

    for G in [int(g) for g in args.worlds.split(",")]:
        r = min(args.rank, G - 1)
        model.aggregator.set_frame_sharding(RankSim(G, r) if G > 1 else None)
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        ops.TIMER = ops.KernelTimer()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.steps):
            step()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.steps
        summ, ops.TIMER = ops.TIMER.summary(), None
        # host submit: the launch sequence of one step started on an idle GPU (the call returns
        # before the kernels finish; with more steps queued behind it the HIP queue back-pressures
        # and the host time reads as the GPU time)
        host = []
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            step()
            host.append((time.perf_counter() - t0) * 1e3)
        torch.cuda.synchronize()
        host_ms = min(host)
        a0, na = shard_range(n, G, r)
        q0, nq = shard_range(n, G, r)
        print(json.dumps({
            "world": G, "rank": r, "views": n, "anchors_local": na, "queries_local": nq,
            "step_ms": round(ms, 2), "host_submit_ms": round(host_ms, 2),
            "expected_views_per_s_at_G": round(n / ms * 1e3, 2),
            "kernel_ms_per_step": {k: round(v["total_ms"] / args.steps, 2)
                                   for k, v in sorted(summ.items(), key=lambda kv: -kv[1]["total_ms"])},
            "kernels": {k: v["kernels"] for k, v in summ.items() if k.startswith("attn")},
        }), flush=True)
    model.aggregator.set_frame_sharding(None)


if __name__ == "__main__":
    main()
