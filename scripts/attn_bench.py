"""Fused attention fwd / fwd+bwd at the ViT-B/16 shape (B 32, T 197, 12 heads x 64): us per call.
Run twice with P2PFL_ATTN_WAVES=4 / 8 to compare block shapes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from p2pfl_amd import ops  # noqa: E402
from p2pfl_amd.ops.fused import attention_qkv  # noqa: E402
from scripts.gemm_bench import timeit  # noqa: E402

ops.ext()
B, T, H = 32, 197, 12
qkv = torch.randn(B, T, 3 * H * 64, device="cuda").to(torch.bfloat16).requires_grad_()
g = torch.randn(B, T, H * 64, device="cuda").to(torch.bfloat16)
fwd = timeit(lambda: attention_qkv(qkv.detach(), H), iters=50)
def fb():
    o = attention_qkv(qkv, H)
    o.backward(g)
both = timeit(fb, iters=50)
fl = 4 * B * H * T * T * 64
print(f"waves={os.environ.get('P2PFL_ATTN_WAVES', '4')}: fwd {fwd * 1e6:.1f} us ({fl / fwd / 1e12:.0f} TF/s), "
      f"fwd+bwd {both * 1e6:.1f} us ({3.5 * fl / both / 1e12:.0f} TF/s)", flush=True)
