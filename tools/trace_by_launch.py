"""Summarise a rocprofv3 kernel trace per (kernel, grid) -- separates the layers of a
benchmark that reuses one kernel for many shapes.

    python tools/trace_by_launch.py gpurun_out/<dir>/run_kernel_trace.csv [filter]
"""
import csv
import sys
from collections import OrderedDict

path = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else ""
groups = OrderedDict()
for r in csv.DictReader(open(path)):
    name = r["Kernel_Name"]
    if filt and filt not in name:
        continue
    key = (name[:70], r["Grid_Size_X"], r["Workgroup_Size_X"])
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    groups.setdefault(key, []).append(d)
for (name, grid, wg), ds in groups.items():
    ds.sort()
    print(f"{name:70s} grid {int(grid)//max(int(wg),1):6d} wg x{len(ds):4d}  median {ds[len(ds)//2]:8.2f} us  min {ds[0]:8.2f}")
