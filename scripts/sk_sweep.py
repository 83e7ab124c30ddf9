"""Stream-K schedule of the ping-pong GEMM on the ViT-B/16 Linear products, vs hipBLASLt
and the data-parallel / split-K configurations of ops.gemm.

    python scripts/sk_sweep.py [--out gpurun_out/sk_sweep.md] [--iters 30] [--check]

For each product: hipBLASLt (torch.mm / F.linear), the best data-parallel or split-K
native configuration, and the stream-K kernel at several grid sizes in both MFMA forms
(HIP-event device time per call, ops/autotune.py's method).  --check compares every
stream-K output with the fp32 product first.
"""

from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from p2pfl_amd.ops import autotune  # noqa: E402
from p2pfl_amd.ops.fused import _fx  # noqa: E402
from p2pfl_amd.ops.gemm import PP, PP_M16, PP_N128, PP_ROWSPLIT, PP_SK, gemm, gemm_reference, sk_iters  # noqa: E402

DP = [(PP | PP_ROWSPLIT | PP_M16, 1), (PP | PP_ROWSPLIT, 1), (PP | PP_N128, 1), (PP | PP_N128 | PP_M16, 1), (PP | PP_M16, 1), (PP, 1), (PP, 2), (PP, 3), (2, 1), (10, 1), (PP, 6), (PP, 8), (PP, 4), (PP, 3), (PP | PP_M16, 6), (10, 6), (4096 | 2, 6)]
GRIDS = (240, 160) if os.environ.get('SK_FULL') is None else (256, 240, 224, 192, 160, 128)


def t_us(fn, iters):
    return autotune._time(fn, iters) * 1e3


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    bf = torch.bfloat16
    torch.manual_seed(0)
    layers = [("qkv", 6304, 768, 2304, False), ("proj", 6304, 768, 768, False), ("fc1", 6304, 768, 3072, True),
              ("fc2", 6304, 3072, 768, False), ("patch", 6272, 768, 768, False)]
    rows = []
    for name, M, K, N, gelu in layers:
        if args.only and args.only not in name:
            continue
        x = torch.randn(M, K, device="cuda").to(bf)
        w = (torch.randn(N, K, device="cuda") * 0.02).to(bf)
        dy = torch.randn(M, N, device="cuda").to(bf)
        bias = torch.randn(N, device="cuda")
        prods = [
            ("fwd", M, N, K, x, w, True, True, bias, gelu,
             (lambda: _fx().bias_gelu_fwd(torch.mm(x, w.t()), bias)) if gelu else (lambda: torch.nn.functional.linear(x, w, bias.to(bf)))),
            ("dgrad", M, K, N, dy, w, True, False, None, False, lambda: torch.mm(dy, w)),
            ("wgrad", N, K, M, dy, x, False, False, None, False, lambda: torch.mm(dy.t(), x)),
        ]
        for kind, m, n, k, a, b, ak, bk, bs, gl, lib in prods:
            fl = 2.0 * m * n * k
            t_lib = t_us(lib, args.iters)
            dp = []
            for v, s in DP:
                if s > 1 and (k // s < 256 or (gl and s > 4)):
                    continue
                try:
                    dp.append((t_us(lambda: gemm(a, b, ak, bk, bias=bs, gelu=gl, want_z=gl, variant=v, splits=s), args.iters), f"v{v} s{s}"))
                except Exception as e:  # noqa: BLE001
                    print(f"skip {name} {kind} v{v} s{s}: {e}", file=sys.stderr)
            dp.sort()
            sk = []
            for m16 in (False, True):
                v = PP | PP_SK | (PP_M16 if m16 else 0)
                for g in GRIDS:
                    if g > sk_iters(m, n, k):
                        continue
                    fn = lambda: gemm(a, b, ak, bk, bias=bs, gelu=gl, want_z=gl, variant=v, splits=g)  # noqa: E731
                    if args.check:
                        out = fn()[0].float()
                        ref = gemm_reference(a, b, ak, bk, bs, gl)[0]
                        err = ((out - ref).abs() / (ref.abs() + 1.0)).max().item()
                        assert err < 3e-2, (name, kind, m16, g, err)
                    sk.append((t_us(fn, args.iters), f"sk{'16' if m16 else ''} g{g}"))
            sk.sort()
            best = min(dp[0], sk[0])
            rows.append((f"{name} {kind}", m, n, k, t_lib, dp[0][0], dp[0][1], sk[0][0], sk[0][1], best[0] / t_lib,
                         fl / best[0] / 1e6, "; ".join(f"{c} {t:.1f}" for t, c in sk[1:5])))
            print(rows[-1], flush=True)
    lines = ["| product | M | N | K | hipBLASLt us | best DP/split-K us | config | best stream-K us | config | best/hipBLASLt | TF/s | next stream-K |",
             "|---|---:|---:|---:|---:|---:|---|---:|---|---:|---:|---|"]
    lines += [f"| {r[0]} | {r[1]} | {r[2]} | {r[3]} | {r[4]:.1f} | {r[5]:.1f} | {r[6]} | {r[7]:.1f} | {r[8]} | {r[9]:.2f} | {r[10]:.0f} | {r[11]} |"
              for r in rows]
    lines.append(f"\nsum over products: hipBLASLt {sum(r[4] for r in rows):.1f} us, best native {sum(min(r[5], r[7]) for r in rows):.1f} us")
    text = "\n".join(lines)
    print(text)
    if args.out:
        os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
        with open(args.out, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
