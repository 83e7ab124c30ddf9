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
