"""Does the chip's clock state (idle vs under sustained load) change which GEMM
path wins a product?  Times hipBLASLt (torch.mm) and the native ping-pong
kernel on the ViT proj input-gradient shape (6304 x 768 x 768) and the qkv
forward shape right after process start (chip idle), then again while
a sustained load of large GEMMs keeps the chip busy between measurements.

    python scripts/dvfs_probe.py
"""

from __future__ import annotations

import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from p2pfl_amd.ops import autotune  # noqa: E402
from p2pfl_amd.ops.gemm import PP, PP_M16, gemm  # noqa: E402


def main() -> None:
    bf = torch.bfloat16
    torch.manual_seed(0)
    dy = torch.randn(6304, 768, device="cuda").to(bf)
    w = (torch.randn(768, 768, device="cuda") * 0.02).to(bf)
    x = torch.randn(6304, 768, device="cuda").to(bf)
    wq = (torch.randn(2304, 768, device="cuda") * 0.02).to(bf)
    big_a = torch.randn(8192, 8192, device="cuda").to(bf)
    cases = {
        "proj dgrad lib": lambda: torch.mm(dy, w),
        "proj dgrad native pp": lambda: gemm(dy, w, True, False, variant=PP),
        "qkv fwd lib": lambda: torch.mm(x, wq.t()),
        "qkv fwd native pp16": lambda: gemm(x, wq, variant=PP | PP_M16),
    }

    def measure(tag: str) -> None:
        row = {k: autotune._time(f, 5) * 1e3 for k, f in cases.items()}
        print(tag + ": " + ", ".join(f"{k} {v:.1f} us" for k, v in row.items()), flush=True)

    measure("cold (first use)")
    measure("cold (second pass)")
    t_end = time.perf_counter() + 3.0
    while time.perf_counter() < t_end:  # sustained load: ~3 s of 8192^3 GEMMs
        for _ in range(10):
            torch.mm(big_a, big_a)
        torch.cuda.synchronize()
    measure("right after 3 s of load")
    for _ in range(20):
        torch.mm(big_a, big_a)
    measure("interleaved with load")
    time.sleep(2.0)
    measure("after 2 s idle")


if __name__ == "__main__":
    main()
