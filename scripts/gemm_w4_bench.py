"""4-wave 256x256 GEMM (variant bit 12, csrc/gemm_w4.hip): numerics vs an fp32
PyTorch reference on every operand layout (tails, split-K in the launch and by
slabs, epilogues), then TF/s vs the 128 tile, the ping-pong kernel and hipBLASLt
on square sizes and the ViT-B/16 products.

    python scripts/gemm_w4_bench.py [--check-only]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from p2pfl_amd import ops  # noqa: E402
from p2pfl_amd.ops.gemm import gemm_reference  # noqa: E402
from p2pfl_amd.ops.splitk import counters, slab_elems, tiles_of  # noqa: E402
from scripts.gemm_bench import timeit  # noqa: E402

C = ops.ext()
bf = torch.bfloat16
PP, W4 = 2048, 4096


def check(M, N, K, ak, bk, splits=1, bias=False, gelu=False, residual=False, out_dtype=bf, slabs=False):
    a = (torch.randn(M, K) if ak else torch.randn(K, M)).cuda().to(bf)
    b = (torch.randn(N, K) if bk else torch.randn(K, N)).cuda().to(bf)
    bi = torch.randn(N, device="cuda") if bias else None
    res = torch.randn(M, N, device="cuda").to(bf) if residual else None
    out = torch.empty(M, N, device="cuda", dtype=out_dtype)
    z = torch.empty(M, N, device="cuda", dtype=bf) if gelu else None
    if splits > 1 and slabs:
        ws = torch.empty(splits * slab_elems(M, N, W4), device="cuda")
        C.gemm(a, b, ak, bk, ws, None, False, None, None, splits, W4)
        C.tile_slab_reduce(ws, splits, M, N, out, W4)
    else:
        ws = cn = None
        if splits > 1:
            ws = torch.empty(splits * slab_elems(M, N, W4), device="cuda")
            cn = counters(tiles_of(M, N), out.device)
        C.gemm(a, b, ak, bk, out, bi, gelu, z, res, splits, W4, ws, cn)
    ref, zr = gemm_reference(a, b, ak, bk, bi, gelu, res)
    torch.cuda.synchronize()
    err = (out.float() - ref).abs().max().item()
    scale = ref.abs().max().item() + 1e-6
    ok = err <= 2e-2 * scale + 1e-2
    if gelu:
        ez = (z.float() - zr).abs().max().item()
        ok = ok and ez <= 2e-2 * (zr.abs().max().item() + 1e-6)
    print(f"check M={M} N={N} K={K} a_kmajor={ak} b_kmajor={bk} splits={splits}{' slabs' if slabs else ''} bias={bias} "
          f"gelu={gelu} res={residual} out={out_dtype}: max|err| {err:.3g} (scale {scale:.3g}) {'OK' if ok else 'FAIL'}",
          flush=True)
    return ok


def main():
    ok = True
    for ak, bk in ((True, True), (True, False), (False, True), (False, False)):
        ok &= check(512, 512, 256, ak, bk)
        ok &= check(296, 264, 128, ak, bk)  # M / N tails, 2 K-tiles
        ok &= check(1000, 776, 64 * 7, ak, bk)  # odd K-tile count
        ok &= check(264, 520, 200, ak, bk) if not (ak or bk) else True  # K tail (m/n-major)
    ok &= check(6304, 768, 768, True, True, bias=True, residual=True)
    ok &= check(6304, 3072, 768, True, True, bias=True, gelu=True)
    ok &= check(6304, 768, 3072, True, False)
    ok &= check(768, 768, 6304, False, False, splits=4)
    ok &= check(768, 3072, 6304, False, False, splits=3, out_dtype=torch.float32)
    ok &= check(768, 2304, 6304, False, False, splits=8, slabs=True, out_dtype=torch.float32)
    ok &= check(256, 256, 64, True, True)
    ok &= check(8, 8, 64, True, True)
    print("ALL OK" if ok else "SOME FAILED", flush=True)
    if not ok or "--check-only" in sys.argv:
        sys.exit(0 if ok else 1)

    print("| shape | v10 (128) | v2048 (ping-pong) | v4096 (4-wave) | hipBLASLt |")
    print("|---|---:|---:|---:|---:|")
    for n in (4096, 8192):
        a = (torch.rand(n, n, device="cuda") * 2 - 1).to(bf)
        b = (torch.rand(n, n, device="cuda") * 2 - 1).to(bf)
        o = torch.empty(n, n, device="cuda", dtype=bf)
        row = []
        for v in (10, PP, W4):
            t = timeit(lambda: C.gemm(a, b, True, True, o, None, False, None, None, 1, v), iters=20, warm=3)
            row.append(f"{2 * n ** 3 / t / 1e12:.0f}")
        t = timeit(lambda: a @ b.t(), iters=20, warm=3)
        row.append(f"{2 * n ** 3 / t / 1e12:.0f}")
        print(f"| {n}^3 | " + " | ".join(row) + " |", flush=True)

    M = 6304
    for name, K, N in [("qkv", 768, 2304), ("proj", 768, 768), ("fc1", 768, 3072), ("fc2", 3072, 768)]:
        x = (torch.rand(M, K, device="cuda") * 2 - 1).to(bf)
        w = (torch.rand(N, K, device="cuda") * 2 - 1).to(bf)
        dy = (torch.rand(M, N, device="cuda") * 2 - 1).to(bf)
        cases = [
            ("fwd", M, N, K, lambda v, o, s, ws, cn: C.gemm(x, w, True, True, o, None, False, None, None, s, v, ws, cn),
             lambda: x @ w.t()),
            ("dgrad", M, K, N, lambda v, o, s, ws, cn: C.gemm(dy, w, True, False, o, None, False, None, None, s, v, ws, cn),
             lambda: dy @ w),
            ("wgrad", N, K, M, lambda v, o, s, ws, cn: C.gemm(dy, x, False, False, o, None, False, None, None, s, v, ws, cn),
             lambda: dy.t() @ x),
        ]
        for kind, m, n, k, fn, lib in cases:
            out = torch.empty((m, n), device="cuda", dtype=bf)
            row = []
            for v in (10, PP, W4):
                tiles = -(-m // 256) * -(-n // 256) if v >= 64 else -(-m // 128) * -(-n // 128)
                best = None
                for s in (1, 2, 3, 4, 6, 8):
                    if s > 1 and v == PP:
                        break  # (ping-pong split-K: row-major slabs, measured in round 3)
                    if tiles * s > 1024:
                        break
                    ws = torch.empty(s * slab_elems(m, n, v), device="cuda") if s > 1 else None
                    cn = counters(tiles_of(m, n), out.device) if s > 1 else None
                    t = timeit(lambda: fn(v, out, s, ws, cn), iters=30)
                    if best is None or t < best[0]:
                        best = (t, s)
                if best is None:
                    row.append("-")
                    continue
                t, s = best
                row.append(f"{2 * m * n * k / t / 1e12:.0f}" + (f" (s{s})" if s > 1 else ""))
            t = timeit(lib, iters=30)
            row.append(f"{2 * m * n * k / t / 1e12:.0f}")
            print(f"| {name} {kind} {m}x{n}x{k} | " + " | ".join(row) + " |", flush=True)


if __name__ == "__main__":
    main()
