"""Run one convolution product repeatedly (for rocprofv3 counter collection).

    python scripts/conv_one.py [fwd|dgrad|dgrad_auto|wgrad] [N C H O k stride pad]

dgrad_auto runs the autograd's input-gradient path (ops/conv.py dgrad_into: split-K
choice, stride 2 by phase).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from p2pfl_amd import ops  # noqa: E402
from p2pfl_amd.ops.conv import dgrad_into, out_hw  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "fwd"
N, C, H, O, k, s, p = (int(v) for v in (sys.argv[2:9] if len(sys.argv) > 8 else (32, 64, 32, 64, 3, 1, 1)))
bf = torch.bfloat16
x4 = torch.randn(N, H, H, C, device="cuda").to(bf)
w4 = torch.randn(O, k, k, C, device="cuda").to(bf)
OH, OW = out_hw(H, H, (k, k), s, p, 1)
dy4 = torch.randn(N, OH, OW, O, device="cuda").to(bf)
X = ops.ext()
for _ in range(20):
    if kind == "fwd":
        X.conv_fwd(x4, w4, s, p, 1, torch.empty(N, OH, OW, O, device="cuda", dtype=bf), 1, 10)
    elif kind == "dgrad_auto":
        dgrad_into(dy4, w4, s, p, 1, torch.empty(N, H, H, C, device="cuda", dtype=bf))
    elif kind == "dgrad":
        X.conv_dgrad(dy4, w4, s, p, 1, torch.empty(N, H, H, C, device="cuda", dtype=bf), [N, H, H, C], 1, 10)
    else:
        X.conv_wgrad(dy4, x4, k, k, s, p, 1, torch.empty(O, k, k, C, device="cuda", dtype=bf), 1, 2)
torch.cuda.synchronize()
print("done", kind, N, C, H, O, k, s, p)
