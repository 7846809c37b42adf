"""hipBLASLt (torch.mm) on the aggregator GEMM shapes, for comparison with tools/kbench.py gemm."""
import torch

from kbench import timeit

M = 2 * 32 * 1374
for name, (N, K) in {"qkv": (3072, 1024), "proj": (1024, 1024), "fc1": (4096, 1024), "fc2": (1024, 4096)}.items():
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) / 32
    b = torch.randn(N, device="cuda", dtype=torch.bfloat16)
    ms = timeit(lambda: torch.mm(a, w.t()))
    ms2 = timeit(lambda: torch.addmm(b, a, w.t()))
    fl = 2.0 * M * N * K
    print(f"hipblaslt {name:5s} mm {ms:7.3f} ms {fl / ms / 1e9:7.1f} TF/s   addmm {ms2:7.3f} ms {fl / ms2 / 1e9:7.1f} TF/s")
