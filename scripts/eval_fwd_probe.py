"""Forward-only (evaluation) kernels of the fused CNN at 128-row launches: us per kernel.

    python scripts/eval_fwd_probe.py            (P2CNN_CONV2_FWD_LDS=1: the LDS-staged conv2)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from p2pfl_amd import ops  # noqa: E402
from p2pfl_amd.learning.fused_cnn import FEAT, HID, FusedCNNEngine  # noqa: E402
from p2pfl_amd.models import CNN  # noqa: E402
from p2pfl_amd.ops.autotune import _time  # noqa: E402

ops.ext()
dev = torch.device("cuda")
eng = FusedCNNEngine(CNN(seed=1).cuda(), device=dev)
C = eng.C
B, M = 128, 128
g = torch.Generator(device="cuda").manual_seed(0)
x = torch.randint(0, 256, (B, 784), dtype=torch.uint8, device="cuda", generator=g)
y = torch.randint(0, 10, (B,), device="cuda", generator=g)
bf = torch.bfloat16
p1 = torch.zeros(M * 196 * 32, dtype=bf, device=dev)
am1 = torch.zeros(M * 196 * 32, dtype=torch.uint8, device=dev)
a1 = torch.zeros(M * FEAT, dtype=bf, device=dev)
am2 = torch.zeros(M * FEAT, dtype=torch.uint8, device=dev)
slabs = torch.zeros(eng.S1 * M * HID, device=dev)
H = torch.zeros(M * HID, dtype=bf, device=dev)
dH = torch.zeros(M * HID, dtype=bf, device=dev)
dl = torch.zeros(M * 10, device=dev)
stats = torch.zeros(4, device=dev)
ks = {
    "conv1_fwd": lambda: C.conv1_fwd(x, None, eng.params, eng.off, p1, am1, None, B),
    "conv2_fwd": lambda: C.conv2_fwd(p1, eng.w2r, eng.params, eng.off, a1, am2, B, M),
    "gemm_fc1": lambda: C.gemm_skinny(a1, eng.w1bf, slabs, M, HID, FEAT, eng.S1),
    "head": lambda: C.head(slabs, eng.S1, M, eng.params, eng.off, y, None, B, False, H, dH, dl, stats, eng.w2bf),
}
res = {k: round(_time(f, 50) * 1e3, 2) for k, f in ks.items()}
print({"lds_conv2": os.environ.get("P2CNN_CONV2_FWD_LDS", "0"), "us": res}, flush=True)
