"""Where does the BatchNorm-statistics conv epilogue spend its time?

Times, per CIFAR ResNet-18 conv shape (batch 32, bf16 NHWC), the plain forward
conv launch (split-K by tile_slab_reduce, as ops.conv dispatches it) against
``conv_fwd_bn`` (statistics epilogue, split-K reduced in the launch), and a
plain forward with in-launch split-K (the BN launch's split handling without the
statistics).  Run under P2_BN_EPI_MODE=0/1/2 (csrc/gemm.h BnEpi::mode) to
separate the per-tile statistics from the cross-tile reduction.

    P2_BN_EPI_MODE=1 python scripts/bn_epi_probe.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from p2pfl_amd.ops import conv as cv  # noqa: E402
from p2pfl_amd.ops.splitk import counters, slab_elems, tiles_of  # noqa: E402


def timeit(fn, iters=50, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / iters


def main():
    dev = torch.device("cuda")
    res = {"mode": int(os.environ.get("P2_BN_EPI_MODE", "0"))}
    for C, HW in ((64, 32), (128, 16), (256, 8), (512, 4)):
        x4 = torch.randn(32, HW, HW, C, device=dev).to(torch.bfloat16)
        w = (torch.randn(C, C, 3, 3, device=dev) * 0.05).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w4 = w.permute(0, 2, 3, 1)
        bw, bb = torch.ones(C, device=dev), torch.zeros(C, device=dev)
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        nbt = torch.zeros(1, dtype=torch.int64, device=dev)
        rows = 32 * HW * HW
        s = cv.mn_splits(rows, C, 9 * C)
        y4 = torch.empty(32, HW, HW, C, device=dev, dtype=torch.bfloat16)

        def plain():
            cv._run_split(lambda o, s_, ws, cnt: cv._C().conv_fwd(x4, w4, 1, 1, 1, o, s_, cv._V_FWD, ws, cnt),
                          rows, C, s, y4, cv._V_FWD)

        ws = torch.empty(max(s, 1) * slab_elems(rows, C), device=dev) if s > 1 else None
        cnt = counters(tiles_of(rows, C), dev) if s > 1 else None

        def plain_inlaunch():
            cv._C().conv_fwd(x4, w4, 1, 1, 1, y4, s, cv._V_FWD, ws, cnt)

        def fused():
            cv._fwd_bn_launch(x4, w, 1, 1, 1, bw, bb, rm, rv, nbt, 1e-5, 0.1)

        res[f"{C}x{HW}x{HW} s{s}"] = {
            "plain": round(timeit(plain), 2),
            "plain_inlaunch": round(timeit(plain_inlaunch), 2),
            "bn_stats": round(timeit(fused), 2),
        }
    print(json.dumps(res))


if __name__ == "__main__":
    main()
