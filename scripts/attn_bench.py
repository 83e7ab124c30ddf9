"""Fused attention kernel vs PyTorch SDPA at the ViT-B/16 shape (B=32, T=197, H=12, d=64)."""
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from p2pfl_amd import ops  # noqa: E402


def sdpa(qkv, H):
    B, T, C3 = qkv.shape
    C = C3 // 3
    q, k, v = qkv.view(B, T, 3, H, C // H).permute(2, 0, 3, 1, 4)
    return F.scaled_dot_product_attention(q, k, v).transpose(1, 2).reshape(B, T, C)


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


B, T, H = 32, 197, 12
qkv = torch.randn(B, T, 3 * 64 * H, device="cuda", dtype=torch.bfloat16, requires_grad=True)
g = torch.randn(B, T, 64 * H, device="cuda", dtype=torch.bfloat16)
for name, f in (("fused", lambda: ops.attention_qkv(qkv, H)), ("sdpa", lambda: sdpa(qkv, H))):
    with torch.no_grad():
        tf = timeit(f)
    tb = timeit(lambda: f().backward(g))
    print(f"{name:6s} fwd {tf:7.1f} us   fwd+bwd {tb:7.1f} us", flush=True)
