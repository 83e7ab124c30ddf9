"""In-process transport."""

from p2pfl_amd.communication.memory.memory_protocol import (
    InMemoryClient,
    InMemoryCommunicationProtocol,
    InMemoryNeighbors,
    InMemoryServer,
)
from p2pfl_amd.communication.memory.registry import InMemoryRegistry

__all__ = ["InMemoryClient", "InMemoryCommunicationProtocol", "InMemoryNeighbors", "InMemoryServer", "InMemoryRegistry"]
