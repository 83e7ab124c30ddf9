"""Where the GPU idles in a rocprofv3 kernel trace: busy share of a steady-state
window, the idle gaps between consecutive kernels (all queues merged), and the
largest gaps with the kernels on either side.

    python tools/gap_summary.py gpurun_out/<dir>/run_kernel_trace.csv [--window-ms 120] [--top 15] [--out f.md]

A round of the N=1 headline bench is GPU-bound when the gaps add up to little;
a gap after the last kernel of one round and before the first of the next is
host time the device waited for (stage machine, readbacks, enqueue).
"""

from __future__ import annotations

import argparse
import csv


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--window-ms", type=float, default=120.0)
    ap.add_argument("--top", type=int, default=15)
    ap.add_argument("--min-gap-us", type=float, default=5.0)
    ap.add_argument("--out", default=None)
    ap.add_argument("--around", default=None, help="also list the kernels (all queues) around the second-to-last "
                    "launch whose name contains this string, with start offsets and durations")
    ap.add_argument("--span", type=int, default=30, help="kernels listed on each side for --around")
    args = ap.parse_args()
    rows = []
    for r in csv.DictReader(open(args.trace)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    t1 = max(e for _, e, _ in rows)
    lo = t1 - int(args.window_ms * 1e6)
    win = [x for x in rows if x[0] >= lo]
    busy = 0
    cur_s, cur_e = win[0][0], win[0][1]
    gaps = []
    prev_name = win[0][2]
    for s, e, name in win[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append(((s - cur_e) / 1e3, prev_name, name))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
        prev_name = name
    busy += cur_e - cur_s
    span = win[-1][1] - win[0][0]
    big = [g for g in gaps if g[0] >= args.min_gap_us]

    def short(n: str) -> str:
        n = n.split("(")[0].replace("void ", "")
        return n[:70]

    lines = [f"# GPU idle gaps: last {args.window_ms:.0f} ms of `{args.trace}`", "",
             f"- kernels in window: {len(win)}; span {span / 1e6:.2f} ms; busy (any kernel running) {busy / 1e6:.2f} ms "
             f"= {100.0 * busy / span:.1f} %",
             f"- gaps: {len(gaps)} total, {sum(g[0] for g in gaps) / 1e3:.2f} ms; "
             f">= {args.min_gap_us:.0f} us: {len(big)}, {sum(g[0] for g in big) / 1e3:.2f} ms", "",
             "| gap us | after | before |", "|---:|---|---|"]
    for g, a, b in sorted(big, key=lambda x: -x[0])[: args.top]:
        lines.append(f"| {g:.1f} | `{short(a)}` | `{short(b)}` |")
    if args.around:
        hits = [i for i, x in enumerate(rows) if args.around in x[2]]
        if len(hits) >= 2:
            c = hits[-2]
            seg = rows[max(0, c - args.span): c + args.span]
            t0 = seg[0][0]
            lines += ["", f"## kernels around the second-to-last `{args.around}`", "",
                      "| start us | dur us | idle before us | kernel |", "|---:|---:|---:|---|"]
            prev_end = seg[0][0]
            for s_, e_, n_ in seg:
                lines.append(f"| {(s_ - t0) / 1e3:.1f} | {(e_ - s_) / 1e3:.1f} | {max(0, s_ - prev_end) / 1e3:.1f} | `{short(n_)}` |")
                prev_end = max(prev_end, e_)
    text = "\n".join(lines)
    print(text)
    if args.out:
        with open(args.out, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
