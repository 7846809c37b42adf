"""Per-step breakdown of a training-step rocprofv3 kernel-stats CSV by kernel family.

Usage: python tools/train_breakdown.py <run_kernel_stats.csv> <steps in the profiled run>
(e.g. profiles/r04_final_train_kernel_stats.csv 4: kbench train's warmup + 3 timed steps,
one adam_kernel launch each).  Families are matched in order, most specific first (mangled
signatures of several kernels mention sr_gemm_epi)."""
import csv
import re
import sys

CATS = [
    ("attention bwd (dK/dV, dQ, delta)", r"attn_bwd"),
    ("qk-norm + RoPE bwd", r"qk_bwd"),
    ("LayerNorm bwd", r"layernorm_bwd"),
    ("LayerNorm fwd", r"layernorm_kernel"),
    ("colsum (bias / LN-parameter grads)", r"colsum"),
    ("Adam + non-finite check", r"adam|nonfinite"),
    ("transpose / cast / vec_fma (weight refresh, dgrad operands)", r"transpose|cast_bf16|weight_refresh|vec_fma"),
    ("key bounds", r"key_norm|key_box"),
    ("runtime copies / fills", r"rocclr"),
    ("ATen kernels", r"at::native"),
    ("attention fwd", r"attn_bf16|attn_merge|attn_f32"),
    ("wgrad GEMMs + reduce", r"wgrad"),
    ("GEMMs (fwd + dgrad)", r"gemm"),
]


def main(path: str, steps: int) -> None:
    agg = {}
    for r in csv.DictReader(open(path)):
        t = int(r["TotalDurationNs"]) / 1e6 / steps
        cat = next((c for c, pat in CATS if re.search(pat, r["Name"])), "other")
        agg[cat] = agg.get(cat, 0.0) + t
    for c, v in sorted(agg.items(), key=lambda x: -x[1]):
        print(f"{v:8.1f} ms/step  {c}")
    print(f"{sum(agg.values()):8.1f} ms/step  all kernels")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]))
