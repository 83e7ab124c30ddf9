"""Tuning experiment: time GEMM kernel variants (scheduling knobs) on ViT shapes."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from p2pfl_amd import ops
from scripts.gemm_bench import timeit

C = ops.ext()
bf = torch.bfloat16
M = 6304
print("| shape | " + " | ".join(f"v{v}" for v in range(8)) + " |")
for name, K, N in [("proj fwd", 768, 768), ("fc1 fwd", 768, 3072), ("fc2 fwd", 3072, 768), ("qkv fwd", 768, 2304)]:
    x = torch.randn(M, K, device="cuda").to(bf)
    w = torch.randn(N, K, device="cuda").to(bf)
    out = torch.empty(M, N, device="cuda", dtype=bf)
    row = []
    for v in range(8):
        t = timeit(lambda: C.gemm(x, w, True, True, out, None, False, None, None, 1, v), iters=40)
        row.append(f"{2 * M * N * K / t / 1e12:.0f}")
    print(f"| {name} | " + " | ".join(row) + " |", flush=True)
# dgrad / wgrad layouts
for name, K, N in [("fc1 dgrad", 3072, 768), ("fc1 wgrad", 6304, 3072)]:
    pass
