"""Summarise rocprofv3 CSV output as a markdown table.

    python tools/prof_summary.py <kernel_stats.csv> [top]
    python tools/prof_summary.py <kernel_trace.csv> [top] --tail-ms T   # only kernels in the last T ms
                                                                         # of the trace (steady state, no warmup)
"""
import csv
import sys
from collections import defaultdict


def main() -> None:
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    tail = None
    if "--tail-ms" in sys.argv:
        tail = float(sys.argv[sys.argv.index("--tail-ms") + 1])
        args = [a for a in args if a != sys.argv[sys.argv.index("--tail-ms") + 1]]
    path, top = args[0], int(args[1]) if len(args) > 1 else 20
    rows = list(csv.DictReader(open(path)))
    agg = defaultdict(lambda: [0, 0.0])
    if "Start_Timestamp" in rows[0]:
        end = max(int(r["End_Timestamp"]) for r in rows)
        lo = end - tail * 1e6 if tail else 0
        sel = [r for r in rows if int(r["Start_Timestamp"]) >= lo]
        for r in sel:
            a = agg[r["Kernel_Name"]]
            a[0] += 1
            a[1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        span = (end - min(int(r["Start_Timestamp"]) for r in sel)) / 1e6 if sel else 0.0
        hdr = f"window: last {tail} ms of the trace (wall span {span:.2f} ms)" if tail else "whole trace"
    else:
        for r in rows:
            agg[r["Name"]] = [int(r["Calls"]), float(r["TotalDurationNs"])]
        hdr = "whole run (rocprofv3 --stats)"
    tot = sum(v[1] for v in agg.values())
    print(f"{hdr}: kernel time {tot / 1e6:.2f} ms over {sum(v[0] for v in agg.values())} launches\n")
    print("| kernel | calls | total ms | avg us | % |\n|---|---:|---:|---:|---:|")
    for name, (n, ns) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"| `{name[:150]}` | {n} | {ns / 1e6:.3f} | {ns / n / 1e3:.2f} | {100 * ns / tot:.1f} |")


if __name__ == "__main__":
    main()
