"""Sanity point for the MFMA GEMM core: square bf16 GEMMs (random operands) vs hipBLASLt, per schedule variant."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from p2pfl_amd import ops  # noqa: E402
from scripts.gemm_bench import timeit  # noqa: E402

C = ops.ext()
bf = torch.bfloat16
for n in (2048, 4096, 8192):
    a = (torch.rand(n, n, device="cuda") * 2 - 1).to(bf)
    b = (torch.rand(n, n, device="cuda") * 2 - 1).to(bf)
    o = torch.empty(n, n, device="cuda", dtype=bf)
    row = []
    for v in (0, 2, 8, 10):
        t = timeit(lambda: C.gemm(a, b, True, True, o, None, False, None, None, 1, v), iters=20, warm=3)
        row.append(f"v{v} {2 * n ** 3 / t / 1e12:.0f}")
    t = timeit(lambda: a @ b.t(), iters=20, warm=3)
    row.append(f"hipBLASLt {2 * n ** 3 / t / 1e12:.0f}")
    print(f"{n}^3 TF/s: " + ", ".join(row), flush=True)
