"""Tuning experiment: time GEMM kernel variants (scheduling knobs, gemm.h) on the ViT-B/16 Linear shapes.

Columns are TF/s per variant bit pattern: bit0 setprio around the MFMAs,
bit1 A-panel tile order, bit2 no XCD remap, bit3 single LDS buffer.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from p2pfl_amd import ops  # noqa: E402
from p2pfl_amd.ops.gemm import splits_for  # noqa: E402
from scripts.gemm_bench import timeit  # noqa: E402

C = ops.ext()
bf = torch.bfloat16
M = 6304
VARIANTS = [0, 1, 2, 8, 9, 10, 12]
print("| product | " + " | ".join(f"v{v}" for v in VARIANTS) + " |")
print("|---|" + "---:|" * len(VARIANTS))
for name, K, N in [("proj", 768, 768), ("fc1", 768, 3072), ("fc2", 3072, 768), ("qkv", 768, 2304)]:
    x = torch.randn(M, K, device="cuda").to(bf)
    w = torch.randn(N, K, device="cuda").to(bf)
    dy = torch.randn(M, N, device="cuda").to(bf)
    s = splits_for(N, K, M)
    cases = [
        ("fwd", M, N, K, lambda v, o: C.gemm(x, w, True, True, o, None, False, None, None, 1, v), (M, N), bf),
        ("dgrad", M, K, N, lambda v, o: C.gemm(dy, w, True, False, o, None, False, None, None, 1, v), (M, K), bf),
        ("wgrad", N, K, M, lambda v, o: C.gemm(dy, x, False, False, o, None, False, None, None, s, v),
         (s, N, K) if s > 1 else (N, K), torch.float32),
    ]
    for kind, m, n, k, fn, oshape, odt in cases:
        out = torch.empty(oshape, device="cuda", dtype=odt)
        row = []
        for v in VARIANTS:
            t = timeit(lambda: fn(v, out), iters=40)
            row.append(f"{2 * m * n * k / t / 1e12:.0f}")
        print(f"| {name} {kind} | " + " | ".join(row) + " |", flush=True)
