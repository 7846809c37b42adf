#!/usr/bin/env python
"""Per-(kernel, grid) averages of rocprofv3 --pmc counters, dispatch by dispatch.

    python tools/pmc_dispatch.py gpurun_out/pmc_dir [name-filter ...]

Unlike tools/pmc_traffic.py (per kernel name), launches of one kernel at different shapes stay
apart (grid size in the key), so e.g. proj and fc2 (both gemm256_kernel<2>) are reported
separately.  FETCH_SIZE is doubled (gfx950 reports half the bytes of 16-B/lane and LDS-DMA
loads, MI355X_MICROARCH.md "HBM"); both size counters are in KB.  With --kernel-trace in the
same pass, the dispatch durations give the effective clock GRBM_GUI_ACTIVE / 8 / duration.
"""
import collections
import csv
import os
import sys

csv.field_size_limit(1 << 30)


def main():
    d = sys.argv[1]
    filt = sys.argv[2:]
    dur = {}
    kt = os.path.join(d, "run_kernel_trace.csv")
    if os.path.exists(kt):
        for r in csv.DictReader(open(kt)):
            dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    per = collections.defaultdict(dict)
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        k = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
        if filt and not any(f in k for f in filt):
            continue
        key = (k, r.get("Grid_Size", "?"))
        per[r["Dispatch_Id"]]["key"] = key
        per[r["Dispatch_Id"]][r["Counter_Name"]] = per[r["Dispatch_Id"]].get(r["Counter_Name"], 0.0) + float(
            r["Counter_Value"])
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for did, v in per.items():
        key = v.pop("key")
        for c, x in v.items():
            acc[key][c].append(x)
        if did in dur:
            acc[key]["_dur"].append(dur[did])
    for (k, grid), v in sorted(acc.items()):
        out = [f"{k[:40]:40s} grid={grid:>9s} n={len(next(iter(v.values()))):3d}"]
        for c, xs in sorted(v.items()):
            m = sum(xs) / len(xs)
            if c == "FETCH_SIZE":
                out.append(f"fetch {2 * m * 1024 / 1e6:9.1f} MB")
            elif c == "WRITE_SIZE":
                out.append(f"write {m * 1024 / 1e6:9.1f} MB")
            elif c == "_dur":
                out.append(f"dur {m * 1e3:8.3f} ms")
            else:
                out.append(f"{c} {m:.4g}")
        if "GRBM_GUI_ACTIVE" in v and "_dur" in v:
            g = sum(v["GRBM_GUI_ACTIVE"]) / len(v["GRBM_GUI_ACTIVE"])
            t = sum(v["_dur"]) / len(v["_dur"])
            out.append(f"clock {g / 8 / t / 1e9:.3f} GHz")
        print("  ".join(out))


if __name__ == "__main__":
    main()
