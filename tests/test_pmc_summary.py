"""CPU test of scripts/pmc_summary.py on synthetic rocprofv3 CSVs."""

from __future__ import annotations

import csv
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _write(path, header, rows):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(header)
        w.writerows(rows)


def test_pmc_summary_joins_counters_and_durations(tmp_path):
    cc = ["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"]
    kt = ["Dispatch_Id", "Kernel_Name", "Start_Timestamp", "End_Timestamp"]
    k = "void p2cnn::head_kernel(float const*, int)"
    # pass 1: FETCH_SIZE split over two dimensions (summed), 2 dispatches of 10 us
    _write(str(tmp_path / "f" / "run_counter_collection.csv"), cc,
           [[1, k, "FETCH_SIZE", 50], [1, k, "FETCH_SIZE", 50], [2, k, "FETCH_SIZE", 100]])
    _write(str(tmp_path / "f" / "run_kernel_trace.csv"), kt, [[1, k, 0, 10000], [2, k, 0, 10000]])
    # pass 2: WRITE_SIZE + the SQ/GRBM counters
    _write(str(tmp_path / "s" / "run_counter_collection.csv"), cc,
           [[7, k, "WRITE_SIZE", 300], [7, k, "SQ_VALU_MFMA_BUSY_CYCLES", 256 * 100], [7, k, "GRBM_GUI_ACTIVE", 8 * 400]])
    out = subprocess.check_output(
        [sys.executable, os.path.join(ROOT, "scripts", "pmc_summary.py"), str(tmp_path / "f"), str(tmp_path / "s")],
        text=True,
    )
    line = [ln for ln in out.splitlines() if ln.startswith("head_kernel")][0].split()
    # columns: name, dur, FETCH_SIZE, GRBM_GUI_ACTIVE, SQ_VALU_MFMA_BUSY_CYCLES, WRITE_SIZE, GB/s, parked, issue-stall, MFMA busy
    assert line[1] == "10.00"
    # (2 * 100 KB + 300 KB) / 10 us = 50 GB/s
    assert line[-4] == "50"  # then parked, issue-stall (nan: no SQ_WAVE_CYCLES), MFMA busy
    assert line[-1] == "25.0%"
