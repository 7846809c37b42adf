#!/usr/bin/env python
"""Host-side cost of one SailRecon forward: how long the Python / C-ABI launch sequence takes to
return (host submit time) against the step's GPU time, and whether the forward blocks on the GPU.

    python tools/host_overhead.py [views ...]      (default: 32 4)

A host submit time close to the step time means the step waits on a device sync inside the
forward; a submit time far below it means the GPU never starves for launches.  Under frame
sharding at G ranks a rank's GPU time shrinks about G-fold while its launch count does not, so
the submit time at the per-rank view count bounds the strong-scaling step from below.
"""

import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "self-supervise-sfm_amd"))

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    views = [int(v) for v in sys.argv[1:]] or [32, 4]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    model, _ = bench.build_model(dev)
    for n in views:
        g = torch.Generator().manual_seed(n)
        x = torch.rand(n, 3, 518, 518, generator=g)
        images = torch.cat([x, x])[None].to(dev)
        lists = dict(no_reloc_list=list(range(n)), reloc_list=list(range(n, 2 * n)), fix_rank=300)

        def step():
            with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
                return model(images, **lists)
        for _ in range(2):
            step()
        torch.cuda.synchronize()
        sub, tot = [], []
        for _ in range(3):
            t0 = time.perf_counter()
            step()
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            sub.append((t1 - t0) * 1e3)
            tot.append((t2 - t0) * 1e3)
        print(f"views={n:3d} host submit {min(sub):8.2f} ms  step {min(tot):8.2f} ms  "
              f"(submit / step {min(sub) / min(tot):.2f})", flush=True)


if __name__ == "__main__":
    main()
