"""gRPC control plane + RCCL point-to-point weights data plane (one peer per GPU).

The reference pushes pickled weight lists through gRPC unary calls
(``grpc_client.py:102-181``, ``gossiper.py:228-239``).  Here, when both ends
of a weights message are ranks of the same ``torch.distributed`` job, only a
small JSON header travels over gRPC (the same ``send_weights`` RPC of
``node.proto``, payload tagged with a magic prefix); the device-resident flat
parameter arena itself goes GPU->GPU with ``dist.send``/``dist.recv``, which
is RCCL over xGMI on an MI355X node (gloo on CPU).  Everything else --
handshakes, heartbeats, votes, metrics, flooding -- is the plain gRPC
transport, so a dist peer interoperates with ordinary gRPC peers (weights to
non-members fall back to encoded bytes).

Deadlock freedom (RCCL point-to-point needs a matching receive and runs the
operations of one communicator in order):

* every ORDERED pair (src -> dst) has its own 2-rank communicator, so a
  communicator only ever carries one direction;
* a sender holds a per-destination lock across "header RPC, then send", so
  the transfers of one direction are strictly sequential and the receiver
  sees headers in send order;
* a receiver runs one receive thread per source: a header is acknowledged at
  once (the RPC returns), the thread posts the matching receive, then hands
  the arena to the command (add_model / init_model) as a device payload.
  A receive can only wait on a sender that has already sent its header and
  is about to send exactly that tensor, so no wait cycle can form.

Limits: a peer that dies between header and tensor leaves that source's
receive thread blocked (other sources keep flowing); a dropped peer is
otherwise handled by the control plane exactly as in the gRPC transport.
"""

from __future__ import annotations

import json
import queue
import threading
from typing import Any, Callable, Dict, List, Optional, Tuple

import torch
import torch.distributed as dist

from p2pfl_amd.communication.grpc.grpc_protocol import GrpcClient, GrpcCommunicationProtocol, GrpcServer
from p2pfl_amd.communication.messages import WeightsMessage
from p2pfl_amd.learning.arena import FlatParams, ParamLayout, flatten
from p2pfl_amd.management.logger import logger
from p2pfl_amd.utils.lockcheck import make_lock

MAGIC = b"P2FDIST1"


def _is_header(payload: Any) -> bool:
    return isinstance(payload, (bytes, bytearray)) and bytes(payload[: len(MAGIC)]) == MAGIC


class DistDataPlane:
    """Directed 2-rank communicators + per-source receive threads.

    Must be constructed by every rank of the job at the same time (it creates
    process groups collectively and exchanges node addresses).
    """

    def __init__(self, addr: str, device: Optional[torch.device] = None) -> None:
        if not dist.is_initialized():
            raise RuntimeError("DistCommunicationProtocol needs torch.distributed initialised (init_distributed())")
        self.rank, self.world = dist.get_rank(), dist.get_world_size()
        self.backend = dist.get_backend()
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if self.backend == "nccl" else torch.device("cpu")
        self.device = torch.device(device)
        # gloo moves host tensors only: GPU arenas are staged through pinned host memory
        self.staged = self.backend != "nccl" and self.device.type == "cuda"
        # every rank creates every directed group in the same order (collective)
        self._groups: Dict[Tuple[int, int], Any] = {}
        for a in range(self.world):
            for b in range(self.world):
                if a != b:
                    g = dist.new_group([a, b])
                    if self.rank in (a, b):
                        self._groups[(a, b)] = g
        addrs: List[Any] = [None] * self.world
        dist.all_gather_object(addrs, addr)
        self.addr_of = {r: a for r, a in enumerate(addrs)}
        self.rank_of = {a: r for r, a in self.addr_of.items()}
        self._send_locks = {r: make_lock("DistDataPlane._send_lock") for r in range(self.world) if r != self.rank}
        self._recv_q: Dict[int, "queue.Queue"] = {}
        self._recv_threads: Dict[int, threading.Thread] = {}
        self._deliver: Optional[Callable[[WeightsMessage], Optional[str]]] = None
        self._lock = make_lock("DistDataPlane._lock")
        self._stopped = False

    # -- setup -----------------------------------------------------------
    def set_delivery(self, fn: Callable[[WeightsMessage], Optional[str]]) -> None:
        """``fn(weights_message)`` runs the command for a fully received arena."""
        self._deliver = fn

    def _bind_device(self) -> None:
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)

    def _sync(self) -> None:
        if self.device.type == "cuda":
            torch.cuda.current_stream(self.device).synchronize()

    # -- send ------------------------------------------------------------
    def send(self, dst_addr: str, msg: WeightsMessage, send_header: Callable[[WeightsMessage], Optional[str]]) -> Optional[str]:
        """Header over the control plane, then the arena over RCCL; returns the control-plane error, if any."""
        dst = self.rank_of[dst_addr]
        params = msg.weights if isinstance(msg.weights, FlatParams) else flatten(msg.weights, self.device)
        flat = params.flat
        if flat.device != self.device:
            flat = flat.to(self.device)
        header = {
            "src": self.rank,
            "numel": int(flat.numel()),
            "dtype": str(flat.dtype).replace("torch.", ""),
            "layout": params.layout.to_json(),
        }
        hmsg = WeightsMessage(
            source=msg.source,
            round=msg.round,
            weights=MAGIC + json.dumps(header).encode(),
            contributors=list(msg.contributors),
            weight=msg.weight,
            cmd=msg.cmd,
        )
        with self._send_locks[dst]:
            if self._stopped:
                return "dist data plane stopped"
            err = send_header(hmsg)
            if err:
                return err
            self._bind_device()
            with logger.span(msg.source, "rccl_send", dst=dst_addr, nbytes=flat.numel() * flat.element_size()):
                wire = flat.cpu() if self.staged else flat
                dist.send(wire, dst=dst, group=self._groups[(self.rank, dst)])
                self._sync()  # the snapshot must outlive the transfer; also back-pressure
        logger.tracer.count(msg.source, "rccl_bytes_sent", flat.numel() * flat.element_size())
        return None

    # -- receive -----------------------------------------------------------
    def on_header(self, msg: WeightsMessage) -> Optional[str]:
        header = json.loads(bytes(msg.weights[len(MAGIC):]).decode())
        src = int(header["src"])
        with self._lock:
            if self._stopped:  # the sender then skips the data transfer
                return "dist data plane stopped"
            q = self._recv_q.get(src)
            if q is None:
                q = self._recv_q[src] = queue.Queue()
                t = threading.Thread(target=self._recv_loop, args=(src, q), name=f"rccl-recv-{src}", daemon=True)
                self._recv_threads[src] = t
                t.start()
            q.put((msg, header))
        return None

    def _recv_loop(self, src: int, q: "queue.Queue") -> None:
        self._bind_device()
        group = self._groups[(src, self.rank)]
        while True:
            item = q.get()
            if item is None:
                return
            msg, header = item
            dtype = getattr(torch, header["dtype"])
            buf = torch.empty(int(header["numel"]), dtype=dtype, device="cpu" if self.staged else self.device)
            dist.recv(buf, src=src, group=group)
            if self.staged:
                buf = buf.to(self.device)
            self._sync()
            logger.tracer.count(self.addr_of[self.rank], "rccl_bytes_recv", buf.numel() * buf.element_size())
            params = FlatParams.from_flat(buf, ParamLayout.from_json(header["layout"]))
            full = WeightsMessage(msg.source, msg.round, params, list(msg.contributors), msg.weight, msg.cmd)
            if self._deliver is not None and not self._stopped:
                try:
                    self._deliver(full)
                except Exception as e:  # a bad model must not kill the receive thread
                    logger.error(self.addr_of[self.rank], f"dist delivery failed: {e}")

    def stop(self, timeout: float = 10.0) -> None:
        """Refuse new transfers, drain in-flight ones, end the receive threads.

        After this returns no thread of this rank is inside a send/recv, so the
        process group can be destroyed (a destroy racing an in-flight
        point-to-point op aborts the process).
        """
        self._stopped = True
        for lk in self._send_locks.values():  # an in-flight send finishes first
            if lk.acquire(timeout=timeout):
                lk.release()
        with self._lock:
            for q in self._recv_q.values():
                q.put(None)
            threads = list(self._recv_threads.values())
        for t in threads:
            t.join(timeout)


class DistServer(GrpcServer):
    """gRPC server whose weights handler diverts data-plane headers to the receive threads."""

    plane: Optional[DistDataPlane] = None

    def handle_weights(self, msg: WeightsMessage) -> Optional[str]:
        if _is_header(msg.weights):
            if self.plane is None:
                return "dist data plane not running"
            if msg.cmd not in self._commands:
                return f"Unknown command: {msg.cmd}"
            return self.plane.on_header(msg)
        return super().handle_weights(msg)

    def deliver_arena(self, msg: WeightsMessage) -> Optional[str]:
        return super().handle_weights(msg)


class DistClient(GrpcClient):
    plane: Optional[DistDataPlane] = None

    def __init__(self, *a: Any, **kw: Any) -> None:
        super().__init__(*a, **kw)
        self._tls = threading.local()  # destination of the send in progress on this thread

    def _deliver(self, handle: Any, msg: Any) -> Optional[str]:
        plane, target = self.plane, getattr(self._tls, "target", None)
        if (
            plane is not None
            and isinstance(msg, WeightsMessage)
            and not isinstance(msg.weights, (bytes, bytearray))
            and target is not None
            and target in plane.rank_of
        ):
            return plane.send(target, msg, lambda h: super(DistClient, self)._deliver(handle, h))
        return super()._deliver(handle, msg)

    def send(self, nei: str, msg: Any, create_connection: bool = False) -> None:
        self._tls.target = nei
        try:
            super().send(nei, msg, create_connection=create_connection)
        finally:
            self._tls.target = None


class DistCommunicationProtocol(GrpcCommunicationProtocol):
    """Drop-in for :class:`GrpcCommunicationProtocol` in a ``torch.distributed`` job (one node per rank).

    All ranks must construct and ``start()`` their nodes together (the data
    plane is set up collectively).  ``peer_addresses()`` then lists every
    rank's node address, which is what ``connect`` needs.
    """

    client_cls = DistClient
    server_cls = DistServer

    def __init__(self, addr: str = "127.0.0.1", commands=None, device: Optional[torch.device] = None) -> None:
        super().__init__(addr, commands)
        self._device = device
        self._plane: Optional[DistDataPlane] = None

    def supports_device_payloads(self) -> bool:
        return True

    def start(self) -> None:
        super().start()
        self._plane = DistDataPlane(self.addr, self._device)
        self._plane.set_delivery(self._server.deliver_arena)
        self._server.plane = self._plane
        self._client.plane = self._plane

    def stop(self) -> None:
        if self._plane is not None:
            self._plane.stop()
        super().stop()

    def peer_addresses(self) -> Dict[int, str]:
        if self._plane is None:
            raise RuntimeError("protocol not started")
        return dict(self._plane.addr_of)
