"""bench.py driver contract on the CPU: one JSON line, for N=1, for N=2 self-launched
(no torchrun: bench.py starts its own worker processes) and for N=2 under torchrun."""

from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _env():
    return dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="2",
                P2PFL_LOCKCHECK="0")


def _json_lines(out: str):
    return [json.loads(ln) for ln in out.splitlines() if ln.startswith("{")]


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world,launcher", [(1, "self"), (2, "self"), (2, "torchrun")])
def test_bench_json_line(world, launcher):
    args = ["bench.py", "--gpus", str(world), "--steps", "1", "--warmup", "1", "--impl", "torch", "--number-sub", "200",
            "--watchdog", "300"]
    if launcher == "self":
        cmd = [sys.executable] + args
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
               "--master-addr=127.0.0.1", f"--master-port={_free_port()}"] + args
    r = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=560)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout  # rank 0 only
    rec = lines[0]
    assert KEYS <= set(rec)
    assert rec["n_gpus"] == world and rec["steps"] == 1 and rec["scaling"] == "weak"
    assert rec["config"]["parallelism"] == "gossip-p2p"  # full Node stack, gossip over the xGMI transport
    assert rec["value"] > 0 and rec["ms_per_step"] > 0
    # whole-job aggregate: value = per-peer throughput x peers
    assert abs(rec["value"] - rec["samples_per_sec_per_peer"] * world) <= 1e-3 * rec["value"] + 0.2


@pytest.mark.timeout(600)
def test_reference_baseline_script_runs():
    """The reference-equivalent baseline (scripts/reference_baseline.py) still runs."""
    cmd = [sys.executable, "scripts/reference_baseline.py", "--steps", "1", "--warmup", "0", "--number-sub", "200"]
    r = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=560)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _json_lines(r.stdout)[0]
    assert rec["ms_per_round"] > 0 and rec["dtype"] == "fp32"
