"""Where the MFMA GEMM's time goes at 4096^3 / 8192^3: full kernel vs probes (gemm.h variant bits:
16 no stores, 32 no K loop, 128 no DMA after the prologue = MFMA + LDS reads only)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from p2pfl_amd import ops  # noqa: E402
from scripts.gemm_bench import timeit  # noqa: E402

C = ops.ext()
bf = torch.bfloat16
print("| n | base | full TF | +no stores | +no DMA (compute only) | no K loop (us) |")
print("|---|---|---:|---:|---:|---:|")
for n in (4096, 8192):
    a = (torch.rand(n, n, device="cuda") * 2 - 1).to(bf)
    b = (torch.rand(n, n, device="cuda") * 2 - 1).to(bf)
    o = torch.empty(n, n, device="cuda", dtype=bf)
    for base in (2, 64, 2 | 512, 64 | 512):
        row = []
        for extra in (0, 16, 128 | 16):
            t = timeit(lambda: C.gemm(a, b, True, True, o, None, False, None, None, 1, base | extra), iters=20, warm=3)
            row.append(f"{2 * n ** 3 / t / 1e12:.0f}")
        t = timeit(lambda: C.gemm(a, b, True, True, o, None, False, None, None, 1, base | 32), iters=20, warm=3)
        row.append(f"{t * 1e6:.1f}")
        print(f"| {n} | v{base} | " + " | ".join(row) + " |", flush=True)
