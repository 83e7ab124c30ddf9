"""Print a rocprofv3 kernel_stats.csv as a compact table (optionally as markdown)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
md = "--md" in sys.argv
if md:
    print("| kernel | calls | total ms | avg us | % |\n|---|---:|---:|---:|---:|")
for r in rows:
    name = r["Name"].replace("void ", "").replace("p2cnn::", "").split("(")[0][:60]
    tot, avg, pct = float(r["TotalDurationNs"]) / 1e6, float(r["AverageNs"]) / 1e3, float(r["Percentage"])
    if pct < 0.05:
        continue
    if md:
        print(f"| `{name}` | {r['Calls']} | {tot:.2f} | {avg:.2f} | {pct:.1f} |")
    else:
        print(f"{name:60s} calls={r['Calls']:>6s} total_ms={tot:8.2f} avg_us={avg:7.2f} pct={pct:5.1f}")
