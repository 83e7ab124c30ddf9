"""Shared fixtures; registers the ``gpu`` marker (tests needing a real MI355X)."""

from __future__ import annotations

import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# Lock-order checking (race detection) is on for the whole suite unless the
# caller sets P2PFL_LOCKCHECK=0; it must be enabled before any lock is built.
os.environ.setdefault("P2PFL_LOCKCHECK", "1")

from p2pfl_amd.settings import Settings  # noqa: E402
from p2pfl_amd.utils import lockcheck  # noqa: E402
from p2pfl_amd.utils import set_test_settings  # noqa: E402

set_test_settings()
Settings.LOG_LEVEL = os.environ.get("P2PFL_TEST_LOG_LEVEL", "INFO")
Settings.LOG_DIR = os.environ.get("P2PFL_TEST_LOG_DIR", "/tmp/p2pfl_amd_test_logs")
if lockcheck.is_enabled():
    # no exemptions: graph captures hold their locks only while recording
    # (warm-ups run under the shared device gate, step_graph.py), so every
    # tracked lock must stay under the limit
    lockcheck.enable(hold_warn_s=10.0)


@pytest.fixture(autouse=True)
def _no_lock_order_violations(request):
    """Fail a test during which the checker saw a potential deadlock."""
    before = len(lockcheck.violations())
    yield
    if request.node.get_closest_marker("lockcheck_expected"):
        return
    new = lockcheck.violations()[before:]
    if new:
        pytest.fail("lock-order violations:\n" + "\n".join(str(v) for v in new), pytrace=False)


def pytest_terminal_summary(terminalreporter, exitstatus, config):
    """Longest hold per lock class (evidence that no capture stalls the other peers)."""
    if not lockcheck.is_enabled():
        return
    holds = lockcheck.max_holds()
    if not holds:
        return
    terminalreporter.write_sep("-", "lockcheck: longest hold per lock class")
    for cls, (dt, th) in sorted(holds.items(), key=lambda kv: -kv[1][0])[:12]:
        terminalreporter.write_line(f"{dt:9.3f} s  {cls}  ({th})")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real AMD GPU (MI355X) and the native extension")
    config.addinivalue_line("markers", "slow: long-running")
    config.addinivalue_line("markers", "lockcheck_expected: the test provokes lock-order violations on purpose")


def pytest_collection_modifyitems(config, items):
    import torch

    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(params=["memory", "grpc", "xgmi"])
def protocol(request):
    if request.param == "memory":
        from p2pfl_amd.communication.memory import InMemoryCommunicationProtocol

        return InMemoryCommunicationProtocol
    if request.param == "xgmi":
        # node-local control bus + data plane on the strict RCCL-semantics simulator
        from p2pfl_amd.communication.xgmi import XgmiSimNetwork

        return XgmiSimNetwork().protocol
    from p2pfl_amd.communication.grpc import GrpcCommunicationProtocol

    return GrpcCommunicationProtocol
