"""In-process transport (reference ``communication/memory/*``).

Every node of a simulation registers its server in :class:`InMemoryRegistry`;
a send is a direct method call on the receiver's server object, synchronous in
the sender's thread, exactly as in the reference (``memory_client.py:107-153``).

MI355X data plane: weight messages carry device-resident
:class:`~p2pfl_amd.learning.arena.FlatParams` snapshots when
``Settings.DEVICE_PAYLOADS`` is on, so virtual peers sharing one GPU exchange
models by reference (zero copies) and peers on different GPUs of the same
process receive them with a single device-to-device copy over xGMI performed by
the receiving learner.  Nothing is serialised on the host.
"""

from __future__ import annotations

import time
from typing import Any, List, Optional

from p2pfl_amd.commands.command import Command
from p2pfl_amd.communication.client import BaseClient
from p2pfl_amd.communication.memory.registry import InMemoryRegistry
from p2pfl_amd.communication.messages import Message, WeightsMessage
from p2pfl_amd.communication.neighbors import NeighborEntry, Neighbors
from p2pfl_amd.communication.protocol import BaseCommunicationProtocol
from p2pfl_amd.communication.server import ServerCore
from p2pfl_amd.settings import Settings


class InMemoryNeighbors(Neighbors):
    def connect(self, addr: str, non_direct: bool = False, handshake_msg: bool = True) -> NeighborEntry:
        if non_direct:
            return NeighborEntry(None, None, time.time())
        server = InMemoryRegistry.get(addr)
        if server is None or not server.running:
            raise ConnectionError(f"No in-memory node at {addr}")
        if handshake_msg:
            err = server.handshake(self.self_addr)
            if err:
                raise ConnectionError(f"Cannot add a neighbor: {err}")
        return NeighborEntry(None, server, time.time())

    def disconnect(self, addr: str, disconnect_msg: bool = True) -> None:
        try:
            _, server, _ = self.get(addr)
        except KeyError:
            return
        if disconnect_msg and server is not None and server.running:
            server.disconnect(self.self_addr)


class InMemoryClient(BaseClient):
    def _deliver(self, handle: Any, msg: Any) -> Optional[str]:
        if not handle.running:
            raise ConnectionError(f"Node {handle.addr} is down")
        if isinstance(msg, WeightsMessage):
            return handle.send_weights(msg)
        if isinstance(msg, Message):
            return handle.send_message(msg)
        raise TypeError("Message type not supported.")

    def _temporary_handle(self, addr: str) -> Any:
        return InMemoryRegistry.get(addr)


class InMemoryServer(ServerCore):
    def __init__(self, addr: str, gossiper: Any, neighbors: Any, commands: Optional[List[Command]] = None) -> None:
        super().__init__(addr, gossiper, neighbors, commands)
        self.running = False

    def start(self, wait: bool = False) -> None:
        InMemoryRegistry.register(self.addr, self)
        self.running = True

    def stop(self) -> None:
        self.running = False
        InMemoryRegistry.unregister(self.addr, self)

    # transport entry points
    def handshake(self, caller: str) -> Optional[str]:
        return self.handle_handshake(caller)

    def disconnect(self, caller: str) -> None:
        self.handle_disconnect(caller)

    def send_message(self, msg: Message) -> Optional[str]:
        if not self.running:
            raise ConnectionError("server stopped")
        return self.handle_message(msg)

    def send_weights(self, msg: WeightsMessage) -> Optional[str]:
        if not self.running:
            raise ConnectionError("server stopped")
        return self.handle_weights(msg)


class InMemoryCommunicationProtocol(BaseCommunicationProtocol):
    neighbors_cls = InMemoryNeighbors
    client_cls = InMemoryClient
    server_cls = InMemoryServer

    def __init__(self, addr: str = "127.0.0.1", commands: Optional[List[Command]] = None) -> None:
        super().__init__(addr, commands)

    def _resolve_address(self, addr: str) -> str:
        # The Node default address is the gRPC one; in memory every node needs
        # a unique name, so the default gets a fresh one (like gRPC's random port).
        if addr in (None, "", "127.0.0.1"):
            return InMemoryRegistry.fresh_address()
        return addr

    @property
    def supports_device_payloads(self) -> bool:
        return bool(Settings.DEVICE_PAYLOADS)
