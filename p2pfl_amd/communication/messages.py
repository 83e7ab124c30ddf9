"""Transport-neutral message records.

Field sets mirror the reference wire schema (``grpc/proto/node.proto:26-57``):
``Message{source, ttl, hash, cmd, args, round}`` and
``Weights{source, round, weights, contributors, weight, cmd}``.  The in-process
transports pass these objects directly; the gRPC transport converts them to and
from protobuf at the socket edge.

``WeightsMessage.weights`` is either wire bytes (:mod:`p2pfl_amd.learning.wire`)
or, on in-process transports, a device-resident
:class:`~p2pfl_amd.learning.arena.FlatParams` snapshot that never leaves HBM.
"""

from __future__ import annotations

import secrets
from dataclasses import dataclass, field
from typing import Any, Callable, List, Optional


def new_message_hash() -> int:
    """Random signed 63-bit id (the reference used the salted builtin ``hash``)."""
    return secrets.randbits(63)


@dataclass
class Message:
    source: str
    ttl: int
    hash: int
    cmd: str
    args: List[str] = field(default_factory=list)
    round: int = -1


@dataclass
class WeightsMessage:
    source: str
    round: int
    weights: Any
    contributors: List[str] = field(default_factory=list)
    weight: int = 1
    cmd: str = ""
    # Delivery feedback (not on the wire): a transport that learns the fate of a
    # push asynchronously (the xGMI data plane: propose -> ack / decline ->
    # transfer) calls on_result("pending"), then "delivered" or "declined: <why>".
    # Synchronous transports never call it.  See stages/base_node/common.py
    # DeliveryLedger.
    on_result: Optional[Callable[[str], None]] = field(default=None, repr=False, compare=False)

    def nbytes(self) -> int:
        w = self.weights
        if isinstance(w, (bytes, bytearray, memoryview)):
            return len(w)
        return int(getattr(w, "nbytes", 0))
