#!/usr/bin/env python3
"""Per-step launch counts of the training step in its steady state, from a rocprofv3 kernel trace
of `tools/kbench.py train` (run_kernel_trace.csv): the launches between two consecutive Adam
updates (one per step) are one step's.  Runtime copies (__amd_rocclr_copyBuffer), fills
(fillBuffer / ATen FillFunctor) and ATen kernels are counted apart; the one-time work before the
first Adam (model build, flat-parameter packing, workspace allocation) is reported separately.

    python3 tools/train_steady_counts.py gpurun_out/prof_train/run_kernel_trace.csv [out.json]
"""
import bisect
import csv
import json
import sys
from collections import Counter


def kind(name: str) -> str:
    if "copyBuffer" in name:
        return "runtime_copy"
    if "fillBuffer" in name or "FillFunctor" in name:
        return "fill"
    if "at::native" in name:
        return "aten"
    return "own"


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    adam = [int(r["Start_Timestamp"]) for r in rows if "adam_kernel" in r["Kernel_Name"]]
    if len(adam) < 2:
        raise SystemExit("need at least two Adam launches (two steps) in the trace")
    per = [Counter() for _ in range(len(adam) + 1)]
    ms = [0.0] * (len(adam) + 1)
    for r in rows:
        i = bisect.bisect(adam, int(r["Start_Timestamp"]))
        per[i][kind(r["Kernel_Name"])] += 1
        per[i]["launches"] += 1
        ms[i] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    steady = per[1:len(adam)]  # whole steps: between consecutive Adam launches
    out = {"steps": len(steady),
           "per_step": {k: sum(c[k] for c in steady) / len(steady)
                        for k in ("launches", "own", "runtime_copy", "fill", "aten")},
           "kernel_ms_per_step": sum(ms[1:len(adam)]) / len(steady),
           "before_first_step": dict(per[0])}
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 2:
        json.dump(out, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
