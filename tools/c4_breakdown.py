#!/usr/bin/env python3
"""Per-step kernel breakdown of the C4 training step from a rocprofv3 --kernel-trace --stats summary
of `tools/kbench.py train` (1 warmup + SR_TRAIN_STEPS timed steps, every kernel identical per step).

    python3 tools/c4_breakdown.py profiles/r03_train_kernel_stats.csv [steps=4] [step_ms]

Prints one row per kernel (calls / step, ms / step, share of the summed kernel time) and the kernel
families (attention fwd / bwd, GEMM fwd / dgrad / wgrad, LayerNorm, elementwise, ...), so that the
part of the step the KernelTimer tags do not cover is named kernel by kernel."""

import csv
import re
import subprocess
import sys

FAMILIES = [
    ("attention bwd", r"attn_bwd|attention_bwd"),
    ("attention fwd", r"attn_bf16|attn_f32|attn_merge|attention_q"),
    ("GEMM wgrad", r"wgrad"),
    ("GEMM (fwd / dgrad)", r"gemm256|gemm_kernel|splitk_reduce"),
    ("LayerNorm fwd / bwd", r"layernorm|ln_"),
    ("qk-norm / RoPE bwd", r"qk_bwd|rope"),
    ("column sums / reductions", r"colsum|rowdot|reduce"),
    ("optimizer", r"adam|nonfinite"),
    ("loss", r"imc|loss|cdf"),
    ("camera head (fp32 small)", r"small|adaln|silu|pose|act_bwd"),
    ("copies / casts / scatter", r"copy|cast|scatter|transpose|set_special|im2col|fill|memset|elementwise|vec_fma"),
]


def family(name):
    for fam, pat in FAMILIES:
        if re.search(pat, name, re.I):
            return fam
    return "other"


def _targs(enc):
    """Template arguments of an Itanium-mangled anonymous-namespace kernel (the bf16 'DF16b' that
    c++filt does not know, ints, bools, float)."""
    out = []
    for m in re.finditer(r"DF16b|Li(-?\d+)E|Lb([01])E|f|d|i", enc):
        t = m.group(0)
        out.append("bf16" if t == "DF16b" else m.group(1) if m.group(1) is not None else
                   ("true" if m.group(2) == "1" else "false") if m.group(2) is not None else
                   {"f": "float", "d": "double", "i": "int"}[t])
    return out


def demangle(name):
    if not name.startswith("_Z"):
        return name
    m = re.match(r"_ZN12_GLOBAL__N_1(\d+)(\w+)", name)
    if m:
        n = int(m.group(1))
        ident, rest = m.group(2)[:n], m.group(2)[n:]
        if rest.startswith("I"):
            depth, end = 0, 0
            for k, ch in enumerate(rest):
                depth += ch == "I"
                depth -= ch == "E" and not rest[max(0, k - 2):k + 1].startswith(("Li", "Lb"))
            args = _targs(rest[1:rest.find("EEv") + 1] if "EEv" in rest else rest[1:])
            return f"{ident}<{', '.join(args)}>"
        return ident
    try:
        return subprocess.run(["c++filt", name], capture_output=True, text=True, check=True).stdout.strip()
    except (OSError, subprocess.CalledProcessError):
        return name


def short(name):
    # rocprofv3's own demangler prints the bf16 template argument as "bool _Accum"
    name = demangle(name).replace("(anonymous namespace)::", "").replace("bool _Accum", "bf16")
    name = re.sub(r"\((?:[^()]|\([^()]*\))*\)$", "", name)
    return name.replace("void ", "")[:70]


def main():
    path = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    step_ms = float(sys.argv[3]) if len(sys.argv) > 3 else None
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((r["Name"], int(r["Calls"]), int(r["TotalDurationNs"])))
    tot = sum(t for _, _, t in rows) / steps / 1e6
    print(f"summed kernel time {tot:.1f} ms/step over {steps} steps" +
          (f" (step wall time {step_ms:.1f} ms: {step_ms - tot:.1f} ms outside kernels)" if step_ms else ""))
    print("\n| kernel | calls/step | ms/step | share |\n|---|---|---|---|")
    for name, calls, t in sorted(rows, key=lambda r: -r[2]):
        ms = t / steps / 1e6
        if ms < 0.05:
            continue
        print(f"| `{short(name)}` | {calls / steps:g} | {ms:.2f} | {ms / tot:.1%} |")
    fams = {}
    for name, calls, t in rows:
        k = family(demangle(name))
        c, tt = fams.get(k, (0, 0))
        fams[k] = (c + calls, tt + t)
    print("\n| family | calls/step | ms/step | share |\n|---|---|---|---|")
    for k, (c, t) in sorted(fams.items(), key=lambda kv: -kv[1][1]):
        ms = t / steps / 1e6
        print(f"| {k} | {c / steps:g} | {ms:.2f} | {ms / tot:.1%} |")


if __name__ == "__main__":
    main()
