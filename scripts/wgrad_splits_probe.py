"""Weight-gradient split-K factor vs time on the ResNet-18 CIFAR shapes (GPU time, parked stream).

    python scripts/wgrad_splits_probe.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from p2pfl_amd import ops  # noqa: E402
from p2pfl_amd.ops.autotune import _time  # noqa: E402
from p2pfl_amd.ops.conv import _run_split, out_hw, wgrad_splits  # noqa: E402

torch.backends.cudnn.benchmark = True
C_ = ops.ext()
bf = torch.bfloat16
N = 32
SPL = (4, 8, 16, 32, 64)
print("| wgrad | default splits | " + " | ".join(f"s={s}" for s in SPL) + " | MIOpen |")
print("|---|---:|" + "---:|" * (len(SPL) + 1))
for name, C, H, O, k, st, p in [("l1 64x32x32", 64, 32, 64, 3, 1, 1), ("l2 s2 64->128", 64, 32, 128, 3, 2, 1),
                                ("l2 128x16x16", 128, 16, 128, 3, 1, 1), ("l3 s2 128->256", 128, 16, 256, 3, 2, 1),
                                ("l3 256x8x8", 256, 8, 256, 3, 1, 1), ("l4 s2 256->512", 256, 8, 512, 3, 2, 1),
                                ("l4 512x4x4", 512, 4, 512, 3, 1, 1)]:
    x = torch.randn(N, C, H, H, device="cuda").to(bf).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(O, C, k, k, device="cuda") * 0.05).to(bf).contiguous(memory_format=torch.channels_last)
    OH, OW = out_hw(H, H, (k, k), st, p, 1)
    dy = torch.randn(N, O, OH, OW, device="cuda").to(bf).contiguous(memory_format=torch.channels_last)
    x4, dy4 = x.permute(0, 2, 3, 1), dy.permute(0, 2, 3, 1)
    dw4 = torch.empty(O, k, k, C, device="cuda", dtype=bf)
    d = wgrad_splits(O, k * k * C, N * OH * OW)
    row = [str(d)]
    for s in SPL:
        t = _time(lambda: _run_split(lambda o, sp, ws, cnt: C_.conv_wgrad(dy4, x4, k, k, st, p, 1, o, sp, 2, ws, cnt),
                                     O, k * k * C, s, dw4, 2), 30)
        row.append(f"{t * 1e3:.1f}")
    t = _time(lambda: torch.ops.aten.convolution_backward(dy, x, w, None, [st, st], [p, p], [1, 1], False, [0, 0], 1,
                                                          [False, True, False]), 30)
    row.append(f"{t * 1e3:.1f}")
    print(f"| {name} | " + " | ".join(row) + " |", flush=True)
