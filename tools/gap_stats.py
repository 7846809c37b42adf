#!/usr/bin/env python3
"""Idle time between kernels of the steady-state forward, from a rocprofv3 kernel trace of
`bench.py` (run_kernel_trace.csv): each forward starts at the patch-embed GEMM
(gemm256_kernel<4, ...>, one per forward); the gaps (next start - this end, one stream) of the
forwards after the first are summed, bucketed, and the largest are listed with their neighbours.
SR_GAP_BOUNDARY names another once-per-step kernel (adam_kernel for `tools/kbench.py train`).

    python3 tools/gap_stats.py gpurun_out/prof/run_kernel_trace.csv [out.json]
"""
import csv
import json
import os
import re
import sys

BOUNDARY = os.environ.get("SR_GAP_BOUNDARY", "gemm256_kernel<4")


def short(name: str) -> str:
    m = re.search(r"(\w+_kernel(?:<[^()]*>)?)", name)
    return m.group(1) if m else name[:60]


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if BOUNDARY in r["Kernel_Name"]]
    if len(starts) < 3:
        raise SystemExit("need >= 3 forwards in the trace")
    gaps, fwd_ms = [], []
    for a, b in zip(starts[1:-1], starts[2:]):
        t0, t1 = int(rows[a]["Start_Timestamp"]), int(rows[b]["Start_Timestamp"])
        fwd_ms.append((t1 - t0) / 1e6)
        for i in range(a, b):
            g = int(rows[i + 1]["Start_Timestamp"]) - int(rows[i]["End_Timestamp"])
            gaps.append((g, short(rows[i]["Kernel_Name"]), short(rows[i + 1]["Kernel_Name"])))
    nf = len(fwd_ms)
    pos = [g for g, _, _ in gaps if g > 0]
    buckets = {"<2us": 0, "2-5us": 0, "5-10us": 0, "10-50us": 0, ">=50us": 0}
    bsum = dict.fromkeys(buckets, 0.0)
    for g in pos:
        k = "<2us" if g < 2000 else "2-5us" if g < 5000 else "5-10us" if g < 10000 else "10-50us" if g < 50000 else ">=50us"
        buckets[k] += 1
        bsum[k] += g / 1e6
    out = {"forwards": nf, "forward_ms": fwd_ms, "launches_per_forward": len(gaps) / nf,
           "idle_ms_per_forward": sum(pos) / 1e6 / nf,
           "overlap_ms_per_forward": -sum(g for g, _, _ in gaps if g < 0) / 1e6 / nf,
           "gap_count_per_forward": {k: v / nf for k, v in buckets.items()},
           "gap_ms_per_forward": {k: round(v / nf, 3) for k, v in bsum.items()},
           "largest": [{"us": g / 1e3, "after": a, "before": b} for g, a, b in sorted(gaps, reverse=True)[:25]]}
    after = {}
    for g, a, _ in gaps:
        if g > 0:
            after[a] = after.get(a, 0.0) + g / 1e6 / nf
    out["idle_ms_after_kernel"] = dict(sorted(((k, round(v, 3)) for k, v in after.items()), key=lambda kv: -kv[1])[:25])
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
