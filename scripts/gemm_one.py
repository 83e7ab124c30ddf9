"""Run one square GEMM configuration a few times (for rocprofv3 counter passes): gemm_one.py N VARIANT [lib]."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from p2pfl_amd import ops  # noqa: E402

n, v = int(sys.argv[1]), int(sys.argv[2])
C = ops.ext()
a = (torch.rand(n, n, device="cuda") * 2 - 1).to(torch.bfloat16)
b = (torch.rand(n, n, device="cuda") * 2 - 1).to(torch.bfloat16)
o = torch.empty(n, n, device="cuda", dtype=torch.bfloat16)
for _ in range(5):
    if len(sys.argv) > 3:
        torch.matmul(a, b.t(), out=o)
    else:
        C.gemm(a, b, True, True, o, None, False, None, None, 1, v)
torch.cuda.synchronize()
print("ok", flush=True)
