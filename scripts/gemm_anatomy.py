"""Where a native GEMM launch's time goes on the ViT products: the kernel with its
timing-probe variant bits (no C stores / no K loop / no DMA after the prologue),
device time per launch (HIP events behind a spin kernel, as ops/autotune.py
times, so host launch overhead is excluded), next to hipBLASLt.

    python scripts/gemm_anatomy.py [--out gpurun_out/gemm_anatomy.md]

Probe bits: 128-tile kernels (gemm_core.h) bit 4 no stores, bit 5 no K loop,
bit 7 no DMA after the prologue; ping-pong (gemm_pp.hip, bit 11) bit 12 no DMA
after the prologue, bit 13 no stagger, bit 14 no C stores, bit 15 no K loop.
Probe timings are not correct outputs.
"""

from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from p2pfl_amd.ops import autotune  # noqa: E402
from p2pfl_amd.ops.gemm import gemm  # noqa: E402


def dev_time(fn, iters=20) -> float:
    return autotune._time(fn, iters) * 1e3  # us


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    bf = torch.bfloat16
    torch.manual_seed(0)
    shapes = [("qkv fwd", 6304, 2304, 768), ("proj fwd", 6304, 768, 768), ("fc2 fwd", 6304, 768, 3072),
              ("fc1 fwd", 6304, 3072, 768), ("square 4096", 4096, 4096, 4096)]
    kernels = [
        ("pingpong", 2048, {"full": 0, "no stores": 1 << 14, "no K loop": 1 << 15, "no DMA in loop": 1 << 12,
                            "no stagger": 1 << 13}),
        ("pingpong16", 2048 | 65536, {"full": 0, "no stores": 1 << 14, "no K loop": 1 << 15, "no DMA in loop": 1 << 12,
                                      "no stagger": 1 << 13}),
        ("128 dbuf", 2, {"full": 0, "no stores": 16, "no K loop": 32, "no DMA in loop": 128}),
        ("128 1buf", 10, {"full": 0, "no stores": 16, "no K loop": 32}),
        ("128 ring4", 4096 | 2, {"full": 0, "no stores": 16, "no K loop": 32}),
    ]
    lines = ["| product | kernel | " + " | ".join(["full", "no stores", "no K loop", "no DMA in loop", "no stagger"])
             + " | hipBLASLt |", "|---|---|" + "---:|" * 6]
    for name, M, N, K in shapes:
        a = torch.randn(M, K, device="cuda").to(bf)
        b = (torch.randn(N, K, device="cuda") * 0.02).to(bf)
        lib = dev_time(lambda: torch.mm(a, b.t()))
        c = torch.empty(M, N, device="cuda", dtype=bf)
        fill = dev_time(lambda: c.fill_(1.0))
        lines.append(f"| {name} {M}x{N}x{K} | torch fill_ of C ({M * N * 2 / 1e6:.1f} MB) | {fill:.1f} ({M * N * 2 / fill / 1e6:.2f} TB/s) | | | | | |")
        fl = 2.0 * M * N * K
        for kname, v, probes in kernels:
            cells = []
            for col in ["full", "no stores", "no K loop", "no DMA in loop", "no stagger"]:
                if col not in probes:
                    cells.append("-")
                    continue
                t = dev_time(lambda: gemm(a, b, variant=v | probes[col]))
                cells.append(f"{t:.1f}" + (f" ({fl / t / 1e6:.0f} TF)" if col == "full" else ""))
            lines.append(f"| {name} {M}x{N}x{K} | {kname} | " + " | ".join(cells) + f" | {lib:.1f} ({fl / lib / 1e6:.0f} TF) |")
            print(lines[-1], flush=True)
    text = "\n".join(lines)
    print(text)
    if args.out:
        with open(args.out, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
