"""Per-kernel summary of a rocprofv3 rocpd database (``<dir>/*_results.db``).

    python tools/rocpd_summary.py gpurun_out/prof [--top 25] [--last-ms 300] [--md]

Groups the ``kernels`` view by kernel name: calls, total / mean / median
duration; ``--last-ms`` restricts to the last N ms of the trace (steady state).
"""

from __future__ import annotations

import argparse
import glob
import os
import sqlite3
import statistics


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--last-ms", type=float, default=0.0)
    ap.add_argument("--md", action="store_true")
    a = ap.parse_args()
    db = a.path if a.path.endswith(".db") else sorted(glob.glob(os.path.join(a.path, "**", "*.db"), recursive=True))[0]
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name_col = "kernel_name" if "kernel_name" in cols else ("name" if "name" in cols else None)
    rows = list(c.execute(f"select {name_col}, start, end from kernels"))
    if not rows:
        print("no kernels")
        return
    t_end = max(r[2] for r in rows)
    t_beg = min(r[1] for r in rows)
    if a.last_ms:
        rows = [r for r in rows if r[1] >= t_end - a.last_ms * 1e6]
    by: dict = {}
    for n, s, e in rows:
        by.setdefault(n, []).append((e - s) / 1e3)
    total = sum(sum(v) for v in by.values())
    span = (t_end - (t_end - a.last_ms * 1e6 if a.last_ms else t_beg)) / 1e6
    items = sorted(by.items(), key=lambda kv: -sum(kv[1]))[: a.top]
    print(f"kernel time {total / 1e3:.3f} ms over {sum(len(v) for v in by.values())} launches, window {span:.1f} ms")
    if a.md:
        print("\n| kernel | calls | total ms | mean us | median us | % |\n|---|---:|---:|---:|---:|---:|")
    for n, v in items:
        nm = (n[:90] + "...") if len(n) > 93 else n
        if a.md:
            print(f"| `{nm}` | {len(v)} | {sum(v) / 1e3:.3f} | {sum(v) / len(v):.2f} | {statistics.median(v):.2f} | {100 * sum(v) / total:.1f} |")
        else:
            print(f"{len(v):7d} {sum(v) / 1e3:9.3f} ms {sum(v) / len(v):8.2f} us {statistics.median(v):8.2f} us  {nm}")


if __name__ == "__main__":
    main()
