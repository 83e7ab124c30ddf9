"""Why do the Linear autotune timings inside the ViT run differ from the sweep's?

Times hipBLASLt (F.linear with bias) and the native kernels on the ViT proj /
qkv / fc2 forward shapes under the conditions that differ between
scripts/vit_gemm_sweep.py and the in-model ``ops.gemm._plan``: operand values
(randn vs LayerNorm-like activations and 0.02-scaled weights), iteration count
(5 vs 30) and whether the call is preceded by other work.

    python scripts/linear_timing_probe.py
"""

from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from p2pfl_amd.ops import autotune  # noqa: E402
from p2pfl_amd.ops.gemm import PP, PP_M16, gemm  # noqa: E402


def main() -> None:
    bf = torch.bfloat16
    torch.manual_seed(0)
    for name, M, N, K in [("proj", 6304, 768, 768), ("qkv", 6304, 2304, 768), ("fc2", 6304, 768, 3072)]:
        for data in ("randn", "ln"):
            x = torch.randn(M, K, device="cuda")
            if data == "ln":
                x = F.layer_norm(x * 3 + 1, (K,))
            x = x.to(bf)
            w = (torch.randn(N, K, device="cuda") * (0.02 if data == "ln" else 1.0)).to(bf)
            b32 = torch.randn(N, device="cuda") * 0.02
            b16 = b32.to(bf)
            for iters in (5, 30):
                lib = autotune._time(lambda: F.linear(x, w, b16), iters) * 1e3
                nat = autotune._time(lambda: gemm(x, w, bias=b32, variant=PP | PP_M16), iters) * 1e3
                nat32 = autotune._time(lambda: gemm(x, w, bias=b32, variant=PP), iters) * 1e3
                print(f"{name} {M}x{N}x{K} data={data} iters={iters}: hipBLASLt {lib:.1f} us | pp16 {nat:.1f} | pp {nat32:.1f}",
                      flush=True)


if __name__ == "__main__":
    main()
