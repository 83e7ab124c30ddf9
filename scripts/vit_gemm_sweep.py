"""Sweep the native GEMM configurations (variant x split-K) on every ViT-B/16 Linear
product and compare with hipBLASLt (torch.mm) -- the data behind the per-product
choice of ``ops.gemm._plan``.

    python scripts/vit_gemm_sweep.py [--out gpurun_out/vit_gemm_sweep.md] [--iters 30]

Products (M = 32 x 197 = 6304 tokens): forward x.W^T, input gradient dY.W and
weight gradient dY^T.x of qkv (768->2304), proj (768->768), fc1 (768->3072,
with the bias+GELU epilogue), fc2 (3072->768) and the patch embedding
(768->768 over 6272 patches).  Times are HIP-event means over back-to-back
launches (device time, host launch overhead excluded) on random operands;
TF/s dense (2 MNK / t).
"""

from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from p2pfl_amd.ops import autotune  # noqa: E402
from p2pfl_amd.ops.fused import _fx  # noqa: E402
from p2pfl_amd.ops.gemm import gemm  # noqa: E402

VARIANTS = {
    2: "128 dbuf",
    10: "128 1buf",
    4096 | 2: "128 ring4",
    64: "256 dbuf",
    2048: "256 pingpong",
    2048 | 65536: "256 pingpong16",
}
SPLITS = (1, 2, 3, 4, 6, 8)


def timeit(fn, iters: int) -> float:
    """Device time per call in us, host launch overhead excluded (ops/autotune.py's
    method: the stream parked on a spin kernel while every timed call is enqueued)."""
    return autotune._time(fn, iters) * 1e3


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--iters", type=int, default=30)
    args = ap.parse_args()
    bf = torch.bfloat16
    torch.manual_seed(0)
    layers = [("qkv", 6304, 768, 2304, False), ("proj", 6304, 768, 768, False), ("fc1", 6304, 768, 3072, True),
              ("fc2", 6304, 3072, 768, False), ("patch", 6272, 768, 768, False)]
    rows = []
    for name, M, K, N, gelu in layers:
        x = torch.randn(M, K, device="cuda").to(bf)
        w = (torch.randn(N, K, device="cuda") * 0.02).to(bf)
        dy = torch.randn(M, N, device="cuda").to(bf)
        bias = torch.randn(N, device="cuda")
        prods = [
            # (kind, m, n, k, native(variant, splits), library)
            ("fwd", M, N, K, lambda v, s: gemm(x, w, bias=bias, gelu=gelu, want_z=gelu, variant=v, splits=s),
             (lambda: _fx().bias_gelu_fwd(torch.mm(x, w.t()), bias)) if gelu
             else (lambda: torch.nn.functional.linear(x, w, bias.to(bf)))),
            ("dgrad", M, K, N, lambda v, s: gemm(dy, w, True, False, variant=v, splits=s), lambda: torch.mm(dy, w)),
            ("wgrad", N, K, M, lambda v, s: gemm(dy, x, False, False, variant=v, splits=s), lambda: torch.mm(dy.t(), x)),
        ]
        for kind, m, n, k, nat, lib in prods:
            fl = 2.0 * m * n * k
            t_lib = timeit(lib, args.iters)
            res = []
            for v, vname in VARIANTS.items():
                for s in SPLITS:
                    if k // s < 256 or (s > 1 and gelu and kind == "fwd" and s > 4):
                        continue
                    try:
                        t = timeit(lambda: nat(v, s), args.iters)
                    except Exception as e:  # a configuration the bindings refuse
                        print(f"skip {name} {kind} v{v} s{s}: {e}", file=sys.stderr)
                        continue
                    res.append((t, v, s, vname))
            res.sort()
            best = res[0]
            rows.append((f"{name} {kind}", m, n, k, t_lib, fl / t_lib / 1e6, best[0], fl / best[0] / 1e6,
                         f"{best[3]} s{best[2]}", "; ".join(f"{r[3]} s{r[2]} {r[0]:.1f}" for r in res[1:4])))
            print(rows[-1], flush=True)
    head = ("| product | M | N | K | hipBLASLt us | TF/s | best native us | TF/s | config | next best (us) |\n"
            "|---|---:|---:|---:|---:|---:|---:|---:|---|---|")
    lines = [head] + [f"| {r[0]} | {r[1]} | {r[2]} | {r[3]} | {r[4]:.1f} | {r[5]:.0f} | {r[6]:.1f} | {r[7]:.0f} | {r[8]} | {r[9]} |"
                      for r in rows]
    wins = sum(1 for r in rows if r[6] < r[4])
    lines.append(f"\nnative faster on {wins} / {len(rows)} products")
    text = "\n".join(lines)
    print(text)
    if args.out:
        os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
        with open(args.out, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
