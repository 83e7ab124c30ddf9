"""Timing probe: conv forward kernel with parts switched off (variant bits 16: no epilogue stores,
32: no K loop, 64: no loads after the first K-tile, 128: no MFMAs)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from p2pfl_amd import ops  # noqa: E402
from p2pfl_amd.ops.conv import out_hw  # noqa: E402


def t(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    evs = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        evs.append((a, b))
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) * 1e3 for a, b in evs)
    return ts[len(ts) // 2]


X = ops.ext()
bf = torch.bfloat16
for (N, C, H, O, k, s, p) in [(32, 64, 32, 64, 3, 1, 1), (32, 128, 16, 128, 3, 1, 1), (32, 256, 8, 256, 3, 1, 1)]:
    x4 = torch.randn(N, H, H, C, device="cuda").to(bf)
    w4 = torch.randn(O, k, k, C, device="cuda").to(bf)
    OH, OW = out_hw(H, H, (k, k), s, p, 1)
    y = torch.empty(N, OH, OW, O, device="cuda", dtype=bf)
    row = []
    for v in (10, 2, 0, 10 | 32):
        row.append(f"v{v}={t(lambda: X.conv_fwd(x4, w4, s, p, 1, y, 1, v)):.1f}us")
    print(f"N{N} C{C} H{H} O{O}: " + "  ".join(row), flush=True)
# plain GEMM of the same size as l1 (M=32768, N=64, K=576) for comparison
a = torch.randn(32768, 576, device="cuda").to(bf)
b = torch.randn(64, 576, device="cuda").to(bf)
o = torch.empty(32768, 64, device="cuda", dtype=bf)
print("plain gemm 32768x64x576:", "  ".join(f"v{v}={t(lambda: X.gemm(a, b, True, True, o, None, False, None, None, 1, v)):.1f}us" for v in (10, 2, 0, 42)))
print("hipblaslt:", f"{t(lambda: a @ b.t()):.1f}us")
