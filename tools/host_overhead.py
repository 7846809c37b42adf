#!/usr/bin/env python
"""Host-side enqueue time of one forward vs its GPU time (is a small per-rank workload CPU-bound?).

    python tools/host_overhead.py [views ...]

For each N: wall time of step() without synchronising (host: Python + ctypes + launches + the
subsample draws) and with it (GPU), and the number of kernel launches per step.
"""

import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "self-supervise-sfm_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
from sailrecon_amd import ops  # noqa: E402


def main():
    views = [int(v) for v in sys.argv[1:]] or [4, 32]
    dev = torch.device("cuda", 0)
    model, _ = bench.build_model(dev)
    for n in views:
        x = torch.rand(n, 3, 518, 518, generator=torch.Generator().manual_seed(n))
        images = torch.cat([x, x])[None].to(dev)

        def step():
            with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
                return model(images, no_reloc_list=list(range(n)), reloc_list=list(range(n, 2 * n)), fix_rank=300)
        for _ in range(2):
            step()
        torch.cuda.synchronize()
        hs, gs = [], []
        for _ in range(3):
            t0 = time.perf_counter()
            step()
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            hs.append(t1 - t0)
            gs.append(t2 - t0)
        ops.TIMER = ops.KernelTimer()
        step()
        torch.cuda.synchronize()
        launches = sum(len(v) for v in ops.TIMER.records.values())
        ops.TIMER = None
        t0 = time.perf_counter()
        model.aggregator.draw_subsample(24, 1, n, 1369, 300)
        t_draw = time.perf_counter() - t0
        print(f"N={n:3d}: host enqueue {min(hs) * 1e3:7.1f} ms   step wall {min(gs) * 1e3:7.1f} ms   "
              f"tagged launches {launches}   subsample draws {t_draw * 1e3:.1f} ms", flush=True)


if __name__ == "__main__":
    main()
