"""ViT weight-gradient GEMM dW[N,K] = dy[M,N]^T @ x[M,K] (M = 6304): plain mm vs split-K over M.

The output has only 36-144 128x128 tiles for 256 CUs; splitting the 6304-long
reduction into S batches multiplies the parallelism (bmm), then one reduction
of the S fp32 partials.
"""
import time

import torch

M = 32 * 197
dev = "cuda"


def timeit(fn, n=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n


for name, (N, K) in {"qkv": (2304, 768), "proj": (768, 768), "fc1": (3072, 768), "fc2": (768, 3072)}.items():
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    dy = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
    ref = torch.mm(dy.t().float(), x.float())
    res = {"mm": timeit(lambda: torch.mm(dy.t(), x))}
    try:
        o = torch.mm(dy.t(), x, out_dtype=torch.float32)
        res["mm_f32out"] = timeit(lambda: torch.mm(dy.t(), x, out_dtype=torch.float32))
    except Exception as e:  # noqa: BLE001
        print("out_dtype unsupported:", type(e).__name__)
    for S in (2, 4, 8):
        if M % S:
            continue
        def f(S=S):
            p = torch.bmm(dy.view(S, M // S, N).transpose(1, 2), x.view(S, M // S, K))
            return p.sum(0, dtype=torch.float32)
        res[f"bmm{S}+sum"] = timeit(f)
        err = (f().float() - ref).abs().max().item() / ref.abs().max().item()
        res[f"bmm{S}_err"] = err
    e0 = (torch.mm(dy.t(), x).float() - ref).abs().max().item() / ref.abs().max().item()
    line = " ".join(f"{k}={v * 1e6:.1f}us" if not k.endswith("err") else f"{k}={v:.2e}" for k, v in res.items())
    print(f"{name:5s} N={N} K={K} mm_err={e0:.2e} {line}", flush=True)
