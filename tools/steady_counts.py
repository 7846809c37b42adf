"""Steady-state launches per forward from two rocprofv3 --kernel-trace --stats summaries of the same
bench command with different step counts: (calls_B - calls_A) / (steps_B - steps_A)
per kernel name removes the one-time work both runs share (model build, weight packing, the first
forward's bound computations and workspace fills).

    python tools/steady_counts.py A_kernel_stats.csv STEPS_A B_kernel_stats.csv STEPS_B [--json out.json]
"""
import csv
import json
import sys


def load(path):
    return {r["Name"]: (int(r["Calls"]), float(r["TotalDurationNs"])) for r in csv.DictReader(open(path))}


def main():
    a, sa, b, sb = sys.argv[1], int(sys.argv[2]), sys.argv[3], int(sys.argv[4])
    A, B = load(a), load(b)
    d = sb - sa
    rows = []
    for name in sorted(set(A) | set(B)):
        ca, ta = A.get(name, (0, 0.0))
        cb, tb = B.get(name, (0, 0.0))
        calls, ms = (cb - ca) / d, (tb - ta) / d / 1e6
        if calls or abs(ms) > 1e-3:
            rows.append((name, calls, ms))
    rows.sort(key=lambda r: -r[2])
    torch_k = [r for r in rows if "at::native" in r[0] or "at::" in r[0]]
    copies = [r for r in rows if "copyBuffer" in r[0] or "fillBuffer" in r[0]]
    for name, calls, ms in rows:
        print(f"{calls:8.1f} {ms:9.3f} ms  {name[:110]}")
    summary = {"per_forward_total_ms": round(sum(r[2] for r in rows), 3),
               "at_native_kernels_per_forward": round(sum(r[1] for r in torch_k), 1),
               "at_native_ms_per_forward": round(sum(r[2] for r in torch_k), 3),
               "runtime_copies_fills_per_forward": round(sum(r[1] for r in copies), 1),
               "runtime_copies_fills_ms_per_forward": round(sum(r[2] for r in copies), 3),
               "launches_per_forward": round(sum(r[1] for r in rows), 1)}
    print(json.dumps(summary))
    if "--json" in sys.argv:
        out = sys.argv[sys.argv.index("--json") + 1]
        json.dump({"summary": summary, "per_forward": [{"name": n, "calls": c, "ms": round(m, 4)} for n, c, m in rows]},
                  open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
