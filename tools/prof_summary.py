"""Summarise a rocprofv3 --kernel-trace --stats output directory into markdown and drop the raw trace.

    python tools/prof_summary.py gpurun_out/<dir> [--keep-trace] [--top 30]

Writes <dir>.md: kernel-time table (top N by total time), launch count,
total kernel time, and the busy window of the trace; removes
run_kernel_trace.csv unless --keep-trace (traces of whole benchmarks exceed
the gpurun copy-back limit).
"""
import argparse
import csv
import os

ap = argparse.ArgumentParser()
ap.add_argument("dir")
ap.add_argument("--keep-trace", action="store_true")
ap.add_argument("--top", type=int, default=30)
ap.add_argument("--window-ms", type=float, default=0.0, help="also tabulate the last N ms of the trace (steady state)")
args = ap.parse_args()
d = args.dir.rstrip("/")
stats = list(csv.DictReader(open(os.path.join(d, "run_kernel_stats.csv"))))
tot = sum(float(r["TotalDurationNs"]) for r in stats)
calls = sum(int(r["Calls"]) for r in stats)
lines = [f"# rocprofv3 kernel stats: {os.path.basename(d)}", "",
         f"total kernel time {tot / 1e6:.2f} ms over {calls} launches", ""]
trace = os.path.join(d, "run_kernel_trace.csv")
if os.path.exists(trace):
    t0 = t1 = None
    for r in csv.DictReader(open(trace)):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        t0 = s if t0 is None else min(t0, s)
        t1 = e if t1 is None else max(t1, e)
    if t0 is not None:
        lines += [f"trace span {(t1 - t0) / 1e6:.1f} ms", ""]
    if args.window_ms > 0 and t1 is not None:
        lo = t1 - int(args.window_ms * 1e6)
        agg = {}
        for r in csv.DictReader(open(trace)):
            s_, e_ = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if s_ < lo:
                continue
            key = (r["Kernel_Name"], r["Grid_Size_X"])
            agg.setdefault(key, []).append((e_ - s_) / 1e3)
        wt = sum(sum(v) for v in agg.values())
        lines += [f"## steady-state window: last {args.window_ms:.0f} ms -- kernel time {wt / 1e3:.2f} ms, "
                  f"{sum(len(v) for v in agg.values())} launches", "",
                  "| kernel | grid | calls | total ms | median us |", "|---|---:|---:|---:|---:|"]
        for (name, grid), v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[: args.top * 2]:
            v.sort()
            nm = name.replace("|", "/")
            nm = nm[:110] + "..." if len(nm) > 110 else nm
            lines.append(f"| `{nm}` | {grid} | {len(v)} | {sum(v) / 1e3:.3f} | {v[len(v) // 2]:.2f} |")
        lines.append("")
lines += ["| kernel | calls | total ms | avg us | % |", "|---|---:|---:|---:|---:|"]
for r in stats[: args.top]:
    name = r["Name"].replace("|", "/")
    if len(name) > 150:
        name = name[:150] + "..."
    lines.append(f"| `{name}` | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.3f} | "
                 f"{float(r['AverageNs']) / 1e3:.2f} | {float(r['TotalDurationNs']) / tot * 100:.1f} |")
open(d + ".md", "w").write("\n".join(lines) + "\n")
print("\n".join(lines[:40]))
if os.path.exists(trace) and not args.keep_trace:
    os.remove(trace)
