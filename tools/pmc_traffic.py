#!/usr/bin/env python
"""Per-kernel HBM traffic from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE).

    python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write profiles/r02_pmc_traffic.json [views img [fp8]]

Corrections (MI355X_MICROARCH.md, "HBM [CDNA4]"): both counters are in KB;
on gfx950 FETCH_SIZE reports half the bytes of wide coalesced reads (16 B/lane global
and LDS-DMA loads — all of this library's operand loads), so it is doubled; WRITE_SIZE
is exact for 16-B/lane stores.  Output: {kernel: {launches, fetch_bytes, write_bytes,
traffic_bytes}} averaged per launch; bench.py reports ``traffic`` for its dominant
kernel from this file.
"""

import csv
import json
import re
import sys
from collections import defaultdict

csv.field_size_limit(1 << 30)
_NAME = re.compile(r"(\w+_kernel(?:<[^()]*>)?)\(")


def short(name: str) -> str:
    m = _NAME.search(name)
    if m:
        return m.group(1)
    m = re.search(r"_ZN12_GLOBAL__N_1\d+(\w+?_kernel)", name)
    return m.group(1) if m else name[:60]


def per_kernel(path: str, counter: str):
    acc = defaultdict(lambda: [0, 0.0])
    seen = set()
    with open(f"{path}/run_counter_collection.csv") as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != counter:
                continue
            key = (r["Dispatch_Id"], counter)
            if key in seen:
                continue
            seen.add(key)
            a = acc[short(r["Kernel_Name"])]
            a[0] += 1
            a[1] += float(r["Counter_Value"]) * 1024.0
    return acc


def main():
    fetch_dir, write_dir, out = sys.argv[1:4]
    # the bench workload the passes ran (bench.py only quotes traffic for this one)
    views, img = (int(sys.argv[4]), int(sys.argv[5])) if len(sys.argv) > 5 else (32, 518)
    fp8 = sys.argv[6] if len(sys.argv) > 6 else "off"  # bench.py --fp8-global mode of the passes
    fe, wr = per_kernel(fetch_dir, "FETCH_SIZE"), per_kernel(write_dir, "WRITE_SIZE")
    res = {}
    for k in sorted(set(fe) | set(wr)):
        n = max(fe[k][0], wr[k][0])
        fb = 2.0 * fe[k][1] / max(fe[k][0], 1)
        wb = wr[k][1] / max(wr[k][0], 1)
        res[k] = dict(launches=n, fetch_bytes=fb, write_bytes=wb, traffic_bytes=fb + wb)
    with open(out, "w") as f:
        json.dump({"source": [fetch_dir, write_dir], "workload": {"views": views, "img": img, "fp8_global": fp8},
                   "fetch_correction": 2.0, "kernels": res}, f, indent=1)
    for k, v in sorted(res.items(), key=lambda kv: -kv[1]["traffic_bytes"] * kv[1]["launches"])[:15]:
        print(f"{k:45s} n={v['launches']:5d} fetch={v['fetch_bytes'] / 1e6:10.2f} MB write={v['write_bytes'] / 1e6:10.2f} MB")


if __name__ == "__main__":
    main()
