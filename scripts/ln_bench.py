"""LayerNorm kernels at the ViT-B/16 training shape (6304 x 768, bf16): forward
with and without the fused residual add, and the backward, device time per
call (HIP events over back-to-back calls).

    python scripts/ln_bench.py [--reps 200]
"""

from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) * 1000.0 / reps, 2)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    args = ap.parse_args()
    from p2pfl_amd.ops import fused

    N, C = 6304, 768
    x = torch.randn(N, C, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    r = torch.randn(N, C, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    w = torch.randn(C, device="cuda", requires_grad=True)
    b = torch.randn(C, device="cuda", requires_grad=True)
    dy = torch.randn(N, C, device="cuda", dtype=torch.bfloat16)
    res = {}
    with torch.no_grad():
        res["ln_fwd"] = timed(lambda: fused.layer_norm(x, w, b), args.reps)
        res["add_ln_fwd"] = timed(lambda: fused.add_layer_norm(x, r, w, b), args.reps)
    y = fused.layer_norm(x, w, b)
    res["ln_fwd_bwd"] = timed(lambda: torch.autograd.grad(fused.layer_norm(x, w, b), (x, w, b), dy), args.reps)
    out = fused.add_layer_norm(x, r, w, b)
    y2 = out[0] if isinstance(out, tuple) else out
    del y, y2
    res["bytes_ln_fwd_MB"] = round(2 * N * C * 2 / 1e6, 1)
    print(json.dumps({"us_per_call": res}))


if __name__ == "__main__":
    main()
