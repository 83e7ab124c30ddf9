"""gRPC transport (reference ``communication/grpc/*``).

Same service and messages as the reference ``node.proto`` (built at runtime,
see :mod:`.proto`), with the send/receive limits raised to
``Settings.GRPC_MAX_MESSAGE_BYTES`` (reference quirk Q6: the 26 MB MNIST CNN did
not fit gRPC's 4 MiB default).  Weights travel as the safe tensor codec of
:mod:`p2pfl_amd.learning.wire` -- never pickle (Security).

The server uses gRPC's generic handlers instead of generated servicers, and a
pool sized for simulations with many in-process nodes.
"""

from __future__ import annotations

import time
from concurrent import futures
from typing import Any, List, Optional

import grpc

from p2pfl_amd.commands.command import Command
from p2pfl_amd.communication.client import BaseClient
from p2pfl_amd.communication.grpc import proto
from p2pfl_amd.communication.grpc.address import AddressParser
from p2pfl_amd.communication.messages import Message, WeightsMessage
from p2pfl_amd.communication.neighbors import NeighborEntry, Neighbors
from p2pfl_amd.communication.protocol import BaseCommunicationProtocol
from p2pfl_amd.communication.server import ServerCore
from p2pfl_amd.settings import Settings


def _channel_options() -> list:
    n = int(Settings.GRPC_MAX_MESSAGE_BYTES)
    return [("grpc.max_send_message_length", n), ("grpc.max_receive_message_length", n)]


class _Stub:
    """Callable RPC handles on one channel (what protoc would generate)."""

    def __init__(self, channel: grpc.Channel) -> None:
        for name, (req, resp) in proto.METHODS.items():
            setattr(
                self,
                name,
                channel.unary_unary(
                    proto.method_path(name),
                    request_serializer=req.SerializeToString,
                    response_deserializer=resp.FromString,
                ),
            )


# -- message conversion ---------------------------------------------------
def to_proto(msg: Any) -> Any:
    if isinstance(msg, Message):
        return proto.Message(source=msg.source, ttl=msg.ttl, hash=msg.hash, cmd=msg.cmd, args=msg.args, round=msg.round)
    if isinstance(msg, WeightsMessage):
        payload = msg.weights
        if not isinstance(payload, (bytes, bytearray)):
            from p2pfl_amd.learning.wire import encode_params

            payload = encode_params(payload)
        return proto.Weights(
            source=msg.source,
            round=msg.round,
            weights=bytes(payload),
            contributors=msg.contributors,
            weight=msg.weight,
            cmd=msg.cmd,
        )
    raise TypeError("Message type not supported.")


def message_from_proto(p: Any) -> Message:
    return Message(
        source=p.source, ttl=p.ttl, hash=p.hash, cmd=p.cmd, args=list(p.args), round=p.round if p.HasField("round") else -1
    )


def weights_from_proto(p: Any) -> WeightsMessage:
    return WeightsMessage(
        source=p.source, round=p.round, weights=p.weights, contributors=list(p.contributors), weight=p.weight, cmd=p.cmd
    )


# -- neighbours -------------------------------------------------------------
class GrpcNeighbors(Neighbors):
    def connect(self, addr: str, non_direct: bool = False, handshake_msg: bool = True) -> NeighborEntry:
        if non_direct:
            return NeighborEntry(None, None, time.time())
        channel = grpc.insecure_channel(addr, options=_channel_options())
        stub = _Stub(channel)
        if handshake_msg:
            try:
                res = stub.handshake(proto.HandShakeRequest(addr=self.self_addr), timeout=Settings.GRPC_TIMEOUT)
            except Exception:
                channel.close()
                raise
            if res.HasField("error"):
                channel.close()
                raise ConnectionError(f"Cannot add a neighbor: {res.error}")
        return NeighborEntry(channel, stub, time.time())

    def disconnect(self, addr: str, disconnect_msg: bool = True) -> None:
        try:
            channel, stub, _ = self.get(addr)
        except KeyError:
            return
        if disconnect_msg and stub is not None:
            try:
                stub.disconnect(proto.HandShakeRequest(addr=self.self_addr), timeout=Settings.GRPC_TIMEOUT)
            except Exception:
                pass

    def _close_entry(self, entry: NeighborEntry) -> None:
        if entry.conn is not None:
            try:
                entry.conn.close()
            except Exception:
                pass


# -- client -----------------------------------------------------------------
class GrpcClient(BaseClient):
    def _deliver(self, handle: Any, msg: Any) -> Optional[str]:
        if isinstance(msg, WeightsMessage):
            res = handle.send_weights(to_proto(msg), timeout=Settings.GRPC_TIMEOUT)
        elif isinstance(msg, Message):
            res = handle.send_message(to_proto(msg), timeout=Settings.GRPC_TIMEOUT)
        else:
            raise TypeError("Message type not supported.")
        return res.error if res.HasField("error") else None

    def _temporary_handle(self, addr: str) -> Any:
        channel = grpc.insecure_channel(addr, options=_channel_options())
        stub = _Stub(channel)
        stub._channel = channel  # type: ignore[attr-defined]
        return stub

    def _release_temporary(self, handle: Any) -> None:
        ch = getattr(handle, "_channel", None)
        if ch is not None:
            ch.close()


# -- server -----------------------------------------------------------------
class GrpcServer(ServerCore):
    def __init__(self, addr: str, gossiper: Any, neighbors: Any, commands: Optional[List[Command]] = None) -> None:
        super().__init__(addr, gossiper, neighbors, commands)
        self._server: Optional[grpc.Server] = None

    def _handlers(self) -> grpc.GenericRpcHandler:
        def handshake(req, ctx):
            err = self.handle_handshake(req.addr)
            return proto.ResponseMessage(error=err) if err else proto.ResponseMessage()

        def disconnect(req, ctx):
            self.handle_disconnect(req.addr)
            return proto.Empty()

        def send_message(req, ctx):
            err = self.handle_message(message_from_proto(req))
            return proto.ResponseMessage(error=err) if err else proto.ResponseMessage()

        def send_weights(req, ctx):
            err = self.handle_weights(weights_from_proto(req))
            return proto.ResponseMessage(error=err) if err else proto.ResponseMessage()

        impl = {"handshake": handshake, "disconnect": disconnect, "send_message": send_message, "send_weights": send_weights}
        rpcs = {
            name: grpc.unary_unary_rpc_method_handler(
                impl[name], request_deserializer=req.FromString, response_serializer=resp.SerializeToString
            )
            for name, (req, resp) in proto.METHODS.items()
        }
        return grpc.method_handlers_generic_handler(proto.SERVICE, rpcs)

    def start(self, wait: bool = False) -> None:
        self._server = grpc.server(futures.ThreadPoolExecutor(max_workers=8), options=_channel_options())
        self._server.add_generic_rpc_handlers((self._handlers(),))
        try:
            port = self._server.add_insecure_port(self.addr)
        except Exception as e:
            raise Exception(f"Cannot bind the address ({self.addr}): {e}") from e
        if port == 0 and not self.addr.startswith("unix://"):
            raise Exception(f"Cannot bind the address ({self.addr})")
        self._server.start()
        if wait:
            self._server.wait_for_termination()

    def stop(self) -> None:
        if self._server is not None:
            self._server.stop(0)

    def wait_for_termination(self) -> None:
        if self._server is not None:
            self._server.wait_for_termination()


class GrpcCommunicationProtocol(BaseCommunicationProtocol):
    neighbors_cls = GrpcNeighbors
    client_cls = GrpcClient
    server_cls = GrpcServer

    def __init__(self, addr: str = "127.0.0.1", commands: Optional[List[Command]] = None) -> None:
        super().__init__(addr, commands)

    def _resolve_address(self, addr: str) -> str:
        return AddressParser(addr).get_parsed_address()
