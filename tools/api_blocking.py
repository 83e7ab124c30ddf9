"""Which HIP runtime calls block the host: from a rocprofv3 ``--hip-trace`` CSV,
the calls of the last ``--window-ms`` that took longer than ``--min-us``, grouped
by API name (count, total, max), plus the longest ones with their thread id.

    python tools/api_blocking.py gpurun_out/<dir>/run_hip_api_trace.csv [--window-ms 80] [--min-us 100]

A host that runs ahead of the device shows its wait in ONE place per round (the
run-ahead bound); any other long synchronous call (a blocking copy, a pinned
allocation, a device-wide synchronize) drains the device queue and shows up as
an idle gap in the kernel trace (tools/gap_summary.py).
"""

from __future__ import annotations

import argparse
import csv
from collections import defaultdict


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--window-ms", type=float, default=80.0)
    ap.add_argument("--min-us", type=float, default=100.0)
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--out", default=None)
    ap.add_argument("--kernels", default=None, help="kernel-trace CSV: end the window at its last kernel "
                    "(the API trace runs on through teardown)")
    args = ap.parse_args()
    rows = []
    for r in csv.DictReader(open(args.trace)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"], r.get("Thread_Id", "?")))
    t1 = max(e for _, e, _, _ in rows)
    if args.kernels:
        t1 = max(int(r["End_Timestamp"]) for r in csv.DictReader(open(args.kernels)))
    lo = t1 - int(args.window_ms * 1e6)
    win = [x for x in rows if lo <= x[0] <= t1]
    agg = defaultdict(lambda: [0, 0.0, 0.0])
    for s, e, f, _ in win:
        d = (e - s) / 1e3
        a = agg[f]
        a[0] += 1
        a[1] += d
        a[2] = max(a[2], d)
    lines = [f"# HIP API calls, last {args.window_ms:.0f} ms of `{args.trace}` ({len(win)} calls)", "",
             "| API | calls | total us | max us |", "|---|---:|---:|---:|"]
    for f, (n, tot, mx) in sorted(agg.items(), key=lambda kv: -kv[1][1])[: args.top]:
        lines.append(f"| `{f}` | {n} | {tot:.0f} | {mx:.0f} |")
    longc = sorted([x for x in win if (x[1] - x[0]) / 1e3 >= args.min_us], key=lambda x: x[0])
    lines += ["", f"## calls >= {args.min_us:.0f} us, in time order", "", "| t (ms from window start) | API | us | thread |",
              "|---:|---|---:|---|"]
    for s, e, f, tid in longc[: 4 * args.top]:
        lines.append(f"| {(s - lo) / 1e6:.3f} | `{f}` | {(e - s) / 1e3:.0f} | {tid} |")
    text = "\n".join(lines)
    print(text)
    if args.out:
        with open(args.out, "w") as fh:
            fh.write(text + "\n")


if __name__ == "__main__":
    main()
