"""Where a stream-K launch's time goes (csrc/gemm_pp.hip variant bits 18-20): the full
launch, no partial-tile stores, no fix-up loads, neither, and XCD-local partials published
with plain stores (bit 20), next to the data-parallel kernel and hipBLASLt.  Probe
timings are not correct outputs.

    python scripts/sk_anatomy.py [--out gpurun_out/sk_anatomy.md]
"""

from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from p2pfl_amd.ops import autotune  # noqa: E402
from p2pfl_amd.ops.gemm import PP, PP_M16, PP_SK, gemm  # noqa: E402


def t_us(fn, iters=30):
    return autotune._time(fn, iters) * 1e3


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    bf = torch.bfloat16
    shapes = [("fc2 fwd", 6304, 768, 3072, True, True, 224), ("fc1 dgrad", 6304, 768, 3072, True, False, 224),
              ("qkv fwd", 6304, 2304, 768, True, True, 240), ("fc2 dgrad", 6304, 3072, 768, True, False, 240),
              ("proj fwd", 6304, 768, 768, True, True, 160)]
    cols = [("full", 0), ("no part. stores", 1 << 18), ("no fix-up loads", 1 << 19), ("neither", 3 << 18),
            ("local plain st.", 1 << 20), ("no K loop", 1 << 15), ("no K loop, neither", (1 << 15) | (3 << 18))]
    lines = ["| product | grid | " + " | ".join(c for c, _ in cols) + " | DP pingpong | hipBLASLt |",
             "|---|---:|" + "---:|" * (len(cols) + 2)]
    for name, M, N, K, ak, bk, g in shapes:
        a = torch.randn(M, K, device="cuda").to(bf) if ak else torch.randn(K, M, device="cuda").to(bf)
        b = torch.randn(N, K, device="cuda").to(bf) if bk else torch.randn(K, N, device="cuda").to(bf)
        cells = [f"{t_us(lambda: gemm(a, b, ak, bk, variant=PP | PP_SK | bits, splits=g)):.1f}" for _, bits in cols]
        dp = t_us(lambda: gemm(a, b, ak, bk, variant=PP))
        A = a if ak else a.t()
        B = b if bk else b.t()
        lib = t_us(lambda: torch.mm(A, B.t()))
        lines.append(f"| {name} {M}x{N}x{K} | {g} | " + " | ".join(cells) + f" | {dp:.1f} | {lib:.1f} |")
        print(lines[-1], flush=True)
    text = "\n".join(lines)
    print(text)
    if args.out:
        with open(args.out, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
