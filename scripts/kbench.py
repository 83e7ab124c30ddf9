"""Per-kernel micro-benchmark of the fused CNN step (MI355X).

Times every kernel of one training step in isolation (each launched ``--reps``
times back to back, HIP events around the batch) on the engine's real buffers,
after one full warm-up step so every input holds realistic data.  Meant to be
run directly or under ``rocprofv3 --pmc ... -- python3 scripts/kbench.py``.

    python scripts/kbench.py [--reps 200] [--only route,conv_adam]
"""

from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--only", default="")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--no-graph", action="store_true", help="skip the graph-captured step (use under --pmc)")
    args = ap.parse_args()

    from p2pfl_amd.learning.fused_cnn import FusedCNNEngine
    from p2pfl_amd.models import CNN

    dev = torch.device("cuda")
    eng = FusedCNNEngine(CNN(seed=0).to(dev), device=dev)
    C, M, B = eng.C, eng.mrows, args.batch
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randint(0, 256, (B, 1, 28, 28), dtype=torch.uint8, device=dev, generator=g).reshape(-1, 784)
    y = torch.randint(0, 10, (B,), device=dev, generator=g)
    stats = torch.zeros(4, device=dev)
    for _ in range(3):
        eng.train_step_async(x, y, None, B, stats, 1)
    torch.cuda.synchronize()
    a = eng._adam()
    # Adam kernels write into the params: run them on scratch copies so repeated
    # launches do not drift the weights into NaN territory
    P, Mm, V = eng.params.clone(), eng.m.clone(), eng.v.clone()
    w1t = eng.w1bf.view(2048, 3136).t().contiguous()  # for the W1^T-shadow variants
    w2s = torch.zeros(10 * 2048, dtype=torch.bfloat16, device=dev)  # scratch bf16 W2 copy for the Adam arm
    rws = torch.zeros(98 * 2 * M * 32, device=dev)  # split-K routing partials / tickets
    rctr = torch.zeros(98, dtype=torch.int32, device=dev)
    ks = {
        "conv1_fwd": lambda: C.conv1_fwd(x, None, eng.params, eng.off, eng.p1, eng.am1, eng.p1s, B),
        "conv2_fwd": lambda: C.conv2_fwd(eng.p1, eng.w2r, eng.params, eng.off, eng.a1, eng.am2, B, M),
        "conv12_fwd": lambda: C.conv12_fwd(x, None, eng.params, eng.off, eng.w2r, None, eng.am1, eng.p1s, eng.a1, eng.am2, B, M),
        "gemm_fc1": lambda: C.gemm_skinny(eng.a1, eng.w1bf, eng.slabs1, M, 2048, 3136, eng.S1),
        "head": lambda: C.head(eng.slabs1, eng.S1, M, eng.params, eng.off, y, None, B, True, eng.H, eng.dH, eng.dlogits, stats, eng.w2bf),
        "head_w2fp32": lambda: C.head(eng.slabs1, eng.S1, M, eng.params, eng.off, y, None, B, True, eng.H, eng.dH, eng.dlogits, stats),
        "route_fc2": lambda: C.route_fc2(eng.dH, eng.w1_route, eng.am2, M, B, eng.dc2m, eng.gb, eng.dlogits, eng.H, P, Mm, V, None, eng.off, eng.adam_t, 1, *a, True, eng.route_rm),
        "route_dA1_only": lambda: C.route_fc2(eng.dH, eng.w1bf, eng.am2, M, B, eng.dc2m, eng.gb, eng.dlogits, eng.H, P, Mm, V, None, eng.off, eng.adam_t, 1, *a, False, True),
        "route_dA1_split2": lambda: C.route_fc2(eng.dH, eng.w1bf, eng.am2, M, B, eng.dc2m, eng.gb, eng.dlogits, eng.H, P, Mm, V, None, eng.off, eng.adam_t, 1, *a, False, True, rws, rctr),
        "route_dA1_w1t": lambda: C.route_fc2(eng.dH, w1t, eng.am2, M, B, eng.dc2m, eng.gb, eng.dlogits, eng.H, P, Mm, V, None, eng.off, eng.adam_t, 1, *a, False, False),
        "fc1_conv_adam_w1t": lambda: C.fc1_conv_adam(eng.dH, eng.a1, M, eng.wslab1, eng.wslab2, eng.gb, B, P, Mm, V, None, eng.w1bf, w1t, eng.w2r, eng.w2q, eng.off, eng.adam_t, 1, *a, eng.dlogits, eng.H),
        "fc1_conv_adam": lambda: C.fc1_conv_adam(eng.dH, eng.a1, M, eng.wslab1, eng.wslab2, eng.gb, B, P, Mm, V, None, eng.w1bf, eng.w1tbf, eng.w2r, eng.w2q, eng.off, eng.adam_t, 1, *a),
        "fc2_fc1_conv_adam": lambda: C.fc1_conv_adam(eng.dH, eng.a1, M, eng.wslab1, eng.wslab2, eng.gb, B, P, Mm, V, None, eng.w1bf, eng.w1tbf, eng.w2r, eng.w2q, eng.off, eng.adam_t, 1, *a, eng.dlogits, eng.H, w2s),
        "fc1_wgrad_adam": lambda: C.fc1_wgrad_adam(eng.dH, eng.a1, M, P, Mm, V, None, eng.w1bf, eng.w1tbf, eng.off, eng.adam_t, 1, *a),
        "conv2_bwd": lambda: C.conv2_bwd(eng.dc2m, eng.p1s, eng.am1, eng.w2q, x, None, eng.wslab1, eng.wslab2, B),
        "conv_adam": lambda: C.conv_adam(eng.wslab1, eng.wslab2, eng.gb, B, P, Mm, V, None, eng.w2r, eng.w2q, eng.off, eng.adam_t, 1, *a),
    }
    only = [s for s in args.only.split(",") if s]
    res = {}
    for name, fn in ks.items():
        if only and not any(o in name for o in only):
            continue
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        res[name] = round(e0.elapsed_time(e1) * 1000.0 / args.reps, 2)
    # whole step, graph-captured, for reference
    if not only and not args.no_graph:
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            eng.train_step_async(x, y, None, B, stats, 1)
        torch.cuda.current_stream().wait_stream(s)
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            for _ in range(20):
                eng.train_step_async(x, y, None, B, stats, 1)
        gr.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            gr.replay()
        e1.record()
        torch.cuda.synchronize()
        res["step_graph"] = round(e0.elapsed_time(e1) * 1000.0 / 100, 2)
    if not only:
        res["sum_isolated"] = round(sum(v for k, v in res.items() if k in ("conv1_fwd", "conv2_fwd", "gemm_fc1", "head", "route_dA1_split2" if eng.route_ws is not None else "route_dA1_only", "conv2_bwd", "fc2_fc1_conv_adam")), 2)
    print(json.dumps({"us_per_kernel": res, "batch": B}))


if __name__ == "__main__":
    main()
