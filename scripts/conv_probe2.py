"""Where a native convolution's time goes (timing-probe variant bits of csrc/gemm.h), GPU time
with host launch cost hidden; MIOpen with find mode (cudnn.benchmark, as the learner runs it).

    python scripts/conv_probe2.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from p2pfl_amd import ops  # noqa: E402
from p2pfl_amd.ops.autotune import _time  # noqa: E402
from p2pfl_amd.ops.conv import _run_split, mn_splits, out_hw  # noqa: E402

torch.backends.cudnn.benchmark = True
C_ = ops.ext()
bf = torch.bfloat16
N = 32
probes = [(2, "v2"), (2 | 16, "no stores"), (2 | 32, "no K loop"), (2 | 128, "no DMA after prologue"),
          (2 | 32 | 16, "no K loop, no stores"), (4096, "4-stage ring"), (10, "v10 (1 buf)")]
print("| conv fwd | " + " | ".join(n for _, n in probes) + " | v2, in-launch reduction (<= 4 slices) | v2 splits 1 | v2 splits 2 | MIOpen (find) |")
print("|---|" + "---:|" * (len(probes) + 4))
for name, C, H, O, k, s, p in [("l1 64x32x32 3x3", 64, 32, 64, 3, 1, 1), ("l2 128x16x16 3x3", 128, 16, 128, 3, 1, 1),
                               ("l3 256x8x8 3x3", 256, 8, 256, 3, 1, 1), ("l4 512x4x4 3x3", 512, 4, 512, 3, 1, 1),
                               ("l2 s2 64->128", 64, 32, 128, 3, 2, 1)]:
    x = torch.randn(N, C, H, H, device="cuda").to(bf).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(O, C, k, k, device="cuda") * 0.05).to(bf).contiguous(memory_format=torch.channels_last)
    OH, OW = out_hw(H, H, (k, k), s, p, 1)
    x4, w4 = x.permute(0, 2, 3, 1), w.permute(0, 2, 3, 1)
    y4 = torch.empty(N, OH, OW, O, device="cuda", dtype=bf)
    sf = mn_splits(N * OH * OW, O, k * k * C)
    row = []
    for v, _ in probes:
        t = _time(lambda: _run_split(lambda o, sp, ws, cnt: C_.conv_fwd(x4, w4, s, p, 1, o, sp, v, ws, cnt), N * OH * OW, O, sf, y4, v), 30)
        row.append(f"{t * 1e3:.1f}")
    import p2pfl_amd.ops.conv as conv_mod

    keep = conv_mod._CONV_IN_LAUNCH_MAX_SPLITS
    conv_mod._CONV_IN_LAUNCH_MAX_SPLITS = 4  # split-K reduced by the last-arriving slice (<= 4 slices)
    t = _time(lambda: conv_mod._run_split(lambda o, sp, ws, cnt: C_.conv_fwd(x4, w4, s, p, 1, o, sp, 2, ws, cnt), N * OH * OW, O, sf, y4, 2), 30)
    conv_mod._CONV_IN_LAUNCH_MAX_SPLITS = keep
    row.append(f"{t * 1e3:.1f}")
    for s1 in (1, 2):
        t = _time(lambda: conv_mod._run_split(lambda o, sp, ws, cnt: C_.conv_fwd(x4, w4, s, p, 1, o, sp, 2, ws, cnt), N * OH * OW, O, s1, y4, 2), 30)
        row.append(f"{t * 1e3:.1f}")
    t = _time(lambda: torch.nn.functional.conv2d(x, w, None, s, p), 30)
    row.append(f"{t * 1e3:.1f}")
    print(f"| {name} (splits {sf}) | " + " | ".join(row) + " |", flush=True)
