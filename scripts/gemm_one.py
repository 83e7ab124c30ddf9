"""Run one GEMM shape repeatedly (for rocprofv3 counter collection)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from p2pfl_amd import ops
M, N, K = (int(v) for v in (sys.argv[1:4] if len(sys.argv) > 3 else (6304, 768, 3072)))
x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
w = torch.randn(N, K, device="cuda").to(torch.bfloat16)
for _ in range(20):
    ops.gemm(x, w)
torch.cuda.synchronize()
print("done", M, N, K)
