"""Time the hand-written MFMA GEMM against torch.matmul (hipBLASLt) on the ViT-B/16 Linear shapes.

    python scripts/gemm_bench.py [--out profiles/r2_gemm_bench.md]

Shapes: M = 32 x 197 = 6304 tokens; forward x.W^T, input gradient dY.W and
weight gradient dY^T.x of qkv (768->2304), proj (768->768), fc1 (768->3072),
fc2 (3072->768).  TFLOP/s are dense (2 MNK / t); MI355X bf16 dense peak is
about 2.5 PFLOP/s.
"""

from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from p2pfl_amd import ops  # noqa: E402
from p2pfl_amd.ops.gemm import splits_for  # noqa: E402


def timeit(fn, iters=50, warm=10):
    for _ in range(warm):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    M = 6304
    layers = [("qkv", 768, 2304), ("proj", 768, 768), ("fc1", 768, 3072), ("fc2", 3072, 768)]
    rows = []
    bf = torch.bfloat16
    for name, K, N in layers:
        x = torch.randn(M, K, device="cuda").to(bf)
        w = (torch.randn(N, K, device="cuda") * 0.02).to(bf)
        dy = torch.randn(M, N, device="cuda").to(bf)
        cases = [
            ("fwd", M, N, K, lambda: ops.gemm(x, w), lambda: x @ w.t()),
            ("dgrad", M, K, N, lambda: ops.gemm(dy, w, True, False), lambda: dy @ w),
            ("wgrad", N, K, M, lambda: ops.gemm(dy, x, False, False, splits=splits_for(N, K, M)), lambda: dy.t() @ x),
        ]
        for kind, m, n, k, mine, theirs in cases:
            t1, t2 = timeit(mine), timeit(theirs)
            fl = 2.0 * m * n * k
            rows.append((f"{name} {kind}", m, n, k, t1 * 1e6, fl / t1 / 1e12, t2 * 1e6, fl / t2 / 1e12))
    head = "| GEMM | M | N | K | native us | native TF/s | hipBLASLt us | hipBLASLt TF/s |\n|---|---:|---:|---:|---:|---:|---:|---:|"
    lines = [head] + [f"| {r[0]} | {r[1]} | {r[2]} | {r[3]} | {r[4]:.1f} | {r[5]:.0f} | {r[6]:.1f} | {r[7]:.0f} |" for r in rows]
    tot1 = sum(r[4] for r in rows)
    tot2 = sum(r[6] for r in rows)
    lines.append(f"\nsum over the 12 products (one ViT block): native {tot1:.0f} us, hipBLASLt {tot2:.0f} us")
    text = "\n".join(lines)
    print(text, flush=True)
    if args.out:
        with open(args.out, "w") as f:
            f.write("# MFMA GEMM vs hipBLASLt on the ViT-B/16 Linear shapes (MI355X)\n\n")
            f.write("`python scripts/gemm_bench.py`; bf16 operands, fp32 accumulation, bf16 output.\n\n")
            f.write(text + "\n")


if __name__ == "__main__":
    main()
