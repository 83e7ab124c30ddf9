"""Shared fixtures; registers the ``gpu`` marker (tests needing a real MI355X)."""

from __future__ import annotations

import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from p2pfl_amd.settings import Settings  # noqa: E402
from p2pfl_amd.utils import set_test_settings  # noqa: E402

set_test_settings()
Settings.LOG_LEVEL = "INFO"
Settings.LOG_DIR = os.environ.get("P2PFL_TEST_LOG_DIR", "/tmp/p2pfl_amd_test_logs")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real AMD GPU (MI355X) and the native extension")
    config.addinivalue_line("markers", "slow: long-running")


def pytest_collection_modifyitems(config, items):
    import torch

    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(params=["memory", "grpc"])
def protocol(request):
    if request.param == "memory":
        from p2pfl_amd.communication.memory import InMemoryCommunicationProtocol

        return InMemoryCommunicationProtocol
    from p2pfl_amd.communication.grpc import GrpcCommunicationProtocol

    return GrpcCommunicationProtocol
