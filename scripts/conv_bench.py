"""Time the implicit-GEMM convolutions against MIOpen (F.conv2d) on the ResNet-18 CIFAR shapes (GPU time, host launch cost hidden).

    python scripts/conv_bench.py [--batch 32] [--out profiles/r2_conv_bench.md]

Per layer class: forward, input gradient (dgrad) and weight gradient (wgrad,
including its slab reduction), bf16 NHWC, all timed as back-to-back launches.
"""

from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from p2pfl_amd import ops  # noqa: E402
from p2pfl_amd.ops import autotune  # noqa: E402
from p2pfl_amd.ops.autotune import _time  # noqa: E402
from p2pfl_amd.ops.conv import dgrad_into, fwd_into, out_hw, wgrad_into  # noqa: E402


def timeit(fn, iters=30):
    """GPU time per call in seconds: the stream is parked behind a spin kernel while
    the calls are enqueued, so host launch cost (large for the library path) is
    not measured -- as in a replayed HIP graph, where these kernels run."""
    return _time(fn, iters) * 1e-3


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    ops.ext()
    torch.backends.cudnn.benchmark = True  # MIOpen find mode, as the learner runs it
    N = args.batch
    bf = torch.bfloat16
    # (name, C, H, O, k, stride, pad, count in ResNet-18)
    layers = [
        ("l1 3x3", 64, 32, 64, 3, 1, 1, 4),
        ("l2 3x3 s2", 64, 32, 128, 3, 2, 1, 1),
        ("l2 3x3", 128, 16, 128, 3, 1, 1, 3),
        ("l2 sc 1x1 s2", 64, 32, 128, 1, 2, 0, 1),
        ("l3 3x3 s2", 128, 16, 256, 3, 2, 1, 1),
        ("l3 3x3", 256, 8, 256, 3, 1, 1, 3),
        ("l3 sc 1x1 s2", 128, 16, 256, 1, 2, 0, 1),
        ("l4 3x3 s2", 256, 8, 512, 3, 2, 1, 1),
        ("l4 3x3", 512, 4, 512, 3, 1, 1, 3),
        ("l4 sc 1x1 s2", 256, 8, 512, 1, 2, 0, 1),
    ]
    rows = []
    tot_n = tot_m = 0.0
    for name, C, H, O, k, s, p, cnt in layers:
        x = torch.randn(N, C, H, H, device="cuda").to(bf).contiguous(memory_format=torch.channels_last)
        w = (torch.randn(O, C, k, k, device="cuda") * 0.05).to(bf).contiguous(memory_format=torch.channels_last)
        OH, OW = out_hw(H, H, (k, k), s, p, 1)
        dy = torch.randn(N, O, OH, OW, device="cuda").to(bf).contiguous(memory_format=torch.channels_last)
        x4, w4, dy4 = x.permute(0, 2, 3, 1), w.permute(0, 2, 3, 1), dy.permute(0, 2, 3, 1)
        y4 = torch.empty(N, OH, OW, O, device="cuda", dtype=bf)
        dx4 = torch.empty(N, H, H, C, device="cuda", dtype=bf)
        dw4 = torch.empty(O, k, k, C, device="cuda", dtype=bf)
        # the autograd's own entry points: per-shape measured (variant, split-K, stride-2 by phase)
        mine = [
            timeit(lambda: fwd_into(x4, w4, s, p, 1, y4)),
            timeit(lambda: dgrad_into(dy4, w4, s, p, 1, dx4)),
            timeit(lambda: wgrad_into(dy4, x4, s, p, 1, dw4)),
        ]
        xr = x.clone().requires_grad_()
        wr = w.clone().requires_grad_()
        theirs = [
            timeit(lambda: torch.nn.functional.conv2d(x, w, None, s, p)),
            timeit(lambda: torch.ops.aten.convolution_backward(dy, x, w, None, [s, s], [p, p], [1, 1], False, [0, 0], 1, [True, False, False])),
            timeit(lambda: torch.ops.aten.convolution_backward(dy, x, w, None, [s, s], [p, p], [1, 1], False, [0, 0], 1, [False, True, False])),
        ]
        del xr, wr
        fl = 2.0 * N * OH * OW * O * C * k * k
        picked = {key[0]: v for key, (v, _) in autotune.choices().items()
                  if isinstance(key, tuple) and key[0].startswith("conv_") and key[1][1:] == (H, H, C) and key[2:6] == (O, k, k, s)}
        for kind, t1, t2 in zip(("fwd", "dgrad", "wgrad"), mine, theirs):
            rows.append((f"{name} {kind}", cnt, t1 * 1e6, fl / t1 / 1e12, t2 * 1e6, fl / t2 / 1e12,
                         picked.get("conv_" + kind, "-")))
            tot_n += cnt * t1 * 1e6
            tot_m += cnt * t2 * 1e6
    head = ("| conv | x in R18 | native us | native TF/s | MIOpen us | MIOpen TF/s | native config |\n"
            "|---|---:|---:|---:|---:|---:|---|")
    lines = [head] + [f"| {r[0]} | {r[1]} | {r[2]:.1f} | {r[3]:.0f} | {r[4]:.1f} | {r[5]:.0f} | {r[6]} |" for r in rows]
    lines.append(f"\nResNet-18 block convolutions per training step (batch {N}): native {tot_n:.0f} us, MIOpen {tot_m:.0f} us")
    text = "\n".join(lines)
    print(text, flush=True)
    if args.out:
        with open(args.out, "w") as f:
            f.write(f"# Implicit-GEMM convolutions vs MIOpen on ResNet-18 CIFAR shapes (MI355X, batch {N})\n\n")
            f.write("`python scripts/conv_bench.py`; bf16 NHWC, fp32 accumulation.\n\n" + text + "\n")


if __name__ == "__main__":
    main()
