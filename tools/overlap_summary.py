"""How much of one kernel class ran concurrently with another, from a rocprofv3 kernel trace.

    python tools/overlap_summary.py <run_kernel_trace.csv> --a REGEX --b REGEX [--out file.md]

For every kernel matching --a, the time during which at least one kernel
matching --b on a DIFFERENT queue/stream was executing is summed; the report
gives the fraction of A's busy time overlapped that way (cross-stream
concurrency), plus the kernel-time totals.
"""
import argparse
import bisect
import csv
import re

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--a", required=True)
ap.add_argument("--b", required=True)
ap.add_argument("--out", default=None)
args = ap.parse_args()
ra, rb = re.compile(args.a), re.compile(args.b)
A, B = [], []
streams = {}
for r in csv.DictReader(open(args.trace)):
    name = r["Kernel_Name"]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    q = (r.get("Queue_Id"), r.get("Stream_Id"))
    if ra.search(name):
        A.append((s, e, q))
    if rb.search(name):
        B.append((s, e, q))
B.sort()
starts = [b[0] for b in B]
maxdur = max((e - s for s, e, _ in B), default=0)
tot_a = sum(e - s for s, e, _ in A)
ov = 0
for s, e, q in A:
    # union of B kernels on OTHER streams intersecting [s, e)
    lo_i = bisect.bisect_left(starts, s - maxdur)
    hi_i = bisect.bisect_left(starts, e)
    segs = sorted((max(s, bs), min(e, be)) for bs, be, bq in B[lo_i:hi_i] if bq != q and be > s and bs < e)
    cur_s = cur_e = None
    for a, b in segs:
        if cur_e is None or a > cur_e:
            if cur_e is not None:
                ov += cur_e - cur_s
            cur_s, cur_e = a, b
        else:
            cur_e = max(cur_e, b)
    if cur_e is not None:
        ov += cur_e - cur_s
qa = sorted({str(q) for *_, q in A})
qb = sorted({str(q) for *_, q in B})
lines = [
    f"# kernel overlap: A=/{args.a}/ vs B=/{args.b}/", "",
    f"- A: {len(A)} launches, {tot_a / 1e6:.3f} ms busy, on queues/streams {qa}",
    f"- B: {len(B)} launches, {sum(e - s for s, e, _ in B) / 1e6:.3f} ms busy, on queues/streams {qb}",
    f"- A time overlapped by a B kernel on another stream: {ov / 1e6:.3f} ms = {100.0 * ov / max(1, tot_a):.1f} % of A",
]
text = "\n".join(lines)
print(text)
if args.out:
    open(args.out, "w").write(text + "\n")
