"""hipBLASLt rate on the ViT-B/16 training GEMMs (B=32, T=197 -> M=6304), bf16.

    python tools/lab/vit_gemm_bench.py [--tunable]
fwd:   y[M,N]  = x[M,K] @ W[N,K]^T (+ bias)         (F.linear)
dgrad: dx[M,K] = dy[M,N] @ W[N,K]
wgrad: dW[N,K] = dy[M,N]^T @ x[M,K]
"""
import sys
import time

import torch
import torch.nn.functional as F

if "--tunable" in sys.argv:
    sys.path.insert(0, ".")
    from p2pfl_amd.tuning import enable_tuned_gemms

    print("tunable", enable_tuned_gemms())
M = 32 * 197
shapes = {"qkv": (2304, 768), "proj": (768, 768), "fc1": (3072, 768), "fc2": (768, 3072)}
dev = "cuda"
tot = {}
for name, (N, K) in shapes.items():
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
    b = torch.randn(N, device=dev, dtype=torch.bfloat16)
    dy = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
    ops = {
        "fwd": lambda: F.linear(x, w, b),
        "dgrad": lambda: torch.mm(dy, w),
        "wgrad": lambda: torch.mm(dy.t(), x),
    }
    for op, fn in ops.items():
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        n = 50
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / n
        tf = 2 * M * N * K / dt / 1e12
        tot[op] = tot.get(op, 0) + dt
        print(f"{name:5s} {op:6s} M={M} N={N} K={K}: {dt * 1e6:8.1f} us  {tf:7.1f} TFLOP/s", flush=True)
print("per layer (us):", {k: round(v * 1e6, 1) for k, v in tot.items()}, "x12 layers fwd+bwd =", round(sum(tot.values()) * 12e3, 2), "ms/step")
