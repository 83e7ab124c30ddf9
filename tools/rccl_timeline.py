"""Per-round timeline of one rank's kernel trace: when the RCCL transfer kernels, the
FedAvg fold (wsum) and the training epoch ran, relative to each other.

    python tools/rccl_timeline.py <run_kernel_trace.csv> [--out file.md]

An "epoch" is a maximal run of training kernels (p2cnn::) with gaps < --gap-us.  For
every RCCL kernel and FedAvg launch the table says which epoch it overlapped (if any)
and how much of it ran while training kernels of that epoch were executing.
"""
import argparse
import csv
import re

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--out", default=None)
ap.add_argument("--gap-us", type=float, default=400.0)
args = ap.parse_args()
train, other = [], []
for r in csv.DictReader(open(args.trace)):
    name = r["Kernel_Name"]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if "p2cnn::" in name:
        train.append((s, e))
    elif re.search(r"nccl|rccl", name, re.I):
        other.append((s, e, "rccl " + name.split("(")[0][-40:]))
    elif "wsum" in name:
        other.append((s, e, "fedavg wsum"))
train.sort()
epochs = []
for s, e in train:
    if epochs and s - epochs[-1][1] < args.gap_us * 1e3:
        epochs[-1][1] = max(epochs[-1][1], e)
    else:
        epochs.append([s, e])
t0 = min([s for s, _ in train] + [s for s, _, _ in other], default=0)


def busy_in(s, e):
    tot = 0
    for a, b in train:
        if b <= s:
            continue
        if a >= e:
            break
        tot += min(b, e) - max(a, s)
    return tot


lines = [f"# timeline of {args.trace.split('/')[-1]}", "",
         f"- {len(epochs)} training epochs (runs of p2cnn:: kernels), {len(other)} RCCL / FedAvg kernels", ""]
lines.append("| epoch | start ms | end ms |")
lines.append("|---:|---:|---:|")
for i, (s, e) in enumerate(epochs):
    lines.append(f"| {i} | {(s - t0) / 1e6:.3f} | {(e - t0) / 1e6:.3f} |")
lines += ["", "| kernel | start ms | dur us | inside epoch | overlapped by training kernels us |", "|---|---:|---:|---:|---:|"]
tot, ov = 0, 0
for s, e, n in sorted(other):
    ep = next((i for i, (a, b) in enumerate(epochs) if s < b and e > a), None)
    o = busy_in(s, e)
    tot += e - s
    ov += min(o, e - s)
    lines.append(f"| {n} | {(s - t0) / 1e6:.3f} | {(e - s) / 1e3:.1f} | {ep if ep is not None else '-'} | {o / 1e3:.1f} |")
lines.append(f"\nRCCL + FedAvg kernel time {tot / 1e6:.3f} ms, of which {ov / 1e6:.3f} ms ({100.0 * ov / max(tot, 1):.1f} %) "
             f"ran while a training kernel executed")
text = "\n".join(lines)
print(text)
if args.out:
    with open(args.out, "w") as f:
        f.write(text + "\n")
