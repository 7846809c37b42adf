#!/usr/bin/env python
"""One FULL oracle forward of the headline scene (N=32 @518, 64 frames) on the host cores, timed
whole — the check of bench.py's per-layer cpu_baseline estimate at the headline size (VERDICT r3
weak 8), run once on the GPU box's CPU share and committed under profiles/.  No GPU is used.

    python tools/cpu_full.py [--views 32] [--img 518]

Prints a heartbeat every 30 s (the oracle forward takes minutes) and one JSON line at the end:
full-forward seconds, the per-layer estimate on the same host, and their ratio.
"""

import argparse
import json
import os
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "self-supervise-sfm_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--views", type=int, default=32)
    ap.add_argument("--img", type=int, default=518)
    args = ap.parse_args()
    import bench
    t_start = time.perf_counter()
    stop = threading.Event()

    def beat():
        while not stop.wait(30):
            print(f"cpu_full: {time.perf_counter() - t_start:.0f} s elapsed", flush=True)
    threading.Thread(target=beat, daemon=True).start()
    model, phys, logical, threads, note = bench._cpu_threads()
    torch.set_num_threads(threads)
    _, sd = bench.build_model(torch.device("cpu"))
    print(f"cpu_full: {model}, {threads} threads ({note})", flush=True)
    est, parts = bench.cpu_forward_by_layer(sd, args.img, args.views)
    print(f"cpu_full: per-layer estimate {est:.1f} s", flush=True)
    full = bench.cpu_full_forward(sd, args.img, args.views)
    stop.set()
    print(json.dumps({"views": args.views, "img": args.img, "threads": threads, "cpu_model": model,
                      "full_forward_s": round(full, 1), "per_layer_estimate_s": round(est, 1),
                      "estimate_over_full": round(est / full, 3),
                      "views_per_s_full_forward": round(args.views / full, 4),
                      "seconds_per_part": {k: round(v, 3) for k, v in parts.items()}}), flush=True)


if __name__ == "__main__":
    main()
