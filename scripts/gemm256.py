"""Wide-tile (256 x 256, 8 waves; variant bit 6) vs 128 x 128 MFMA GEMM vs hipBLASLt: square sizes and the ViT-B/16 products (TF/s)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from p2pfl_amd import ops  # noqa: E402
from p2pfl_amd.ops.gemm import splits_for  # noqa: E402
from p2pfl_amd.ops.splitk import counters, tiles_of  # noqa: E402
from scripts.gemm_bench import timeit  # noqa: E402

C = ops.ext()
bf = torch.bfloat16
VARS = (10, 2, 258, 64, 65, 322)
print("| shape | v10 (128, 1 buf) | v2 (128, 2 buf) | v258 (128, 2 buf, legacy order) | v64 (256) | v65 (256, setprio) | v322 (256, legacy order) | hipBLASLt |")
print("|---|---:|---:|---:|---:|---:|---:|---:|")
for n in (2048, 4096, 8192):
    a = (torch.rand(n, n, device="cuda") * 2 - 1).to(bf)
    b = (torch.rand(n, n, device="cuda") * 2 - 1).to(bf)
    o = torch.empty(n, n, device="cuda", dtype=bf)
    row = []
    for v in VARS:
        t = timeit(lambda: C.gemm(a, b, True, True, o, None, False, None, None, 1, v), iters=20, warm=3)
        row.append(f"{2 * n ** 3 / t / 1e12:.0f}")
    t = timeit(lambda: a @ b.t(), iters=20, warm=3)
    row.append(f"{2 * n ** 3 / t / 1e12:.0f}")
    print(f"| {n}^3 | " + " | ".join(row) + " |", flush=True)

M = 6304
for name, K, N in [("proj", 768, 768), ("fc1", 768, 3072), ("fc2", 3072, 768), ("qkv", 768, 2304)]:
    x = torch.randn(M, K, device="cuda").to(bf)
    w = torch.randn(N, K, device="cuda").to(bf)
    dy = torch.randn(M, N, device="cuda").to(bf)
    cases = [
        ("fwd", M, N, K, lambda v, o, s, ws, cn: C.gemm(x, w, True, True, o, None, False, None, None, 1, v),
         lambda: x @ w.t()),
        ("dgrad", M, K, N, lambda v, o, s, ws, cn: C.gemm(dy, w, True, False, o, None, False, None, None, 1, v),
         lambda: dy @ w),
        ("wgrad", N, K, M, lambda v, o, s, ws, cn: C.gemm(dy, x, False, False, o, None, False, None, None, s, v, ws, cn),
         lambda: dy.t() @ x),
    ]
    for kind, m, n, k, fn, lib in cases:
        out = torch.empty((m, n), device="cuda", dtype=bf)
        row = []
        for v in VARS:
            s = 1
            if kind == "wgrad":
                s = min(4, splits_for(m, n, k)) if v < 64 else min(4, max(1, 256 // (-(-m // 256) * -(-n // 256))))
            ws = torch.empty(s * m * n, device="cuda") if s > 1 else None
            cn = counters(tiles_of(m, n), out.device) if s > 1 else None
            t = timeit(lambda: fn(v, out, s, ws, cn), iters=40)
            row.append(f"{2 * m * n * k / t / 1e12:.0f}" + (f" (s{s})" if s > 1 else ""))
        t = timeit(lib, iters=40)
        row.append(f"{2 * m * n * k / t / 1e12:.0f}")
        print(f"| {name} {kind} {m}x{n}x{k} | " + " | ".join(row) + " |", flush=True)
