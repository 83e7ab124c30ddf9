"""CLI and bundled examples (reference: p2pfl/cli.py, p2pfl/examples/*)."""

from __future__ import annotations

import os
import socket
import subprocess
import sys

import pytest
from typer.testing import CliRunner

from p2pfl_amd.cli import app, available_examples

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_experiment_list_shows_examples():
    ex = available_examples()
    assert {"mnist", "node1", "node2"} <= set(ex)
    assert all(desc for desc in ex.values())
    res = CliRunner().invoke(app, ["experiment", "list"])
    assert res.exit_code == 0 and "mnist" in res.output


def test_experiment_run_unknown_fails():
    res = CliRunner().invoke(app, ["experiment", "run", "no_such_example"])
    assert res.exit_code == 1


def test_placeholders_and_info():
    r = CliRunner()
    for cmd in ("login", "remote", "launch"):
        assert r.invoke(app, [cmd]).exit_code == 0
    res = r.invoke(app, ["info"])
    assert res.exit_code == 0 and "torch" in res.output


def test_mnist_example_in_process():
    from p2pfl_amd.examples.mnist import mnist

    nodes = mnist(2, 1, 1, show_metrics=False, model="mlp", protocol="memory", device="cpu")
    for n in nodes:
        assert n.state.round is None
        assert n.state.learner.evaluate()["test_metric"] > 0.5


@pytest.mark.timeout(240)
def test_node1_node2_over_grpc():
    """The two-terminal example: node1 waits, node2 connects and runs learning."""
    p1, p2 = _free_port(), _free_port()
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    n1 = subprocess.Popen([sys.executable, "-m", "p2pfl_amd.examples.node1", str(p1), "--timeout", "180"], env=env,
                          stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    try:
        line = n1.stdout.readline()
        assert "listening" in line, line
        out = subprocess.run([sys.executable, "-m", "p2pfl_amd.examples.node2", str(p2), str(p1), "--rounds", "1"],
                             env=env, capture_output=True, text=True, timeout=200)
        assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
        assert "node2 finished" in out.stdout
    finally:
        n1.terminate()
        n1.wait(timeout=30)
