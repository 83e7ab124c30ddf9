"""xGMI transport: one federated peer per GPU of a machine.

``XgmiCommunicationProtocol`` is a drop-in :class:`CommunicationProtocol`
(same 14 methods as the reference's ``GrpcCommunicationProtocol``,
``grpc_communication_protocol.py:35-230``) for peers that live on the GPUs of
one MI355X node:

* **control plane** -- every command message, handshake, heartbeat and vote is
  a msgpack record on the node-local :mod:`bus <p2pfl_amd.communication.xgmi.bus>`
  (abstract ``AF_UNIX`` sockets, microseconds per message, instant detection
  of a dead peer process);
* **data plane** -- a weights message whose payload is a device-resident
  flat arena snapshot becomes a ``wput`` header on the bus plus an RCCL
  transfer over xGMI, scheduled by :class:`~.data_plane.XgmiDataPlane`
  (epoch-grouped, link-parallel, deadlock-free, fault-aware).  The receiver
  checks *before* any byte moves whether its aggregator would accept the model
  (``Command.precheck``), so unneeded partial aggregates cost one header, not a
  full transfer.

Semantics kept from the reference: a failed send or an error reply drops the
neighbour (``grpc_client.py:159-179``, quirk Q13); flooding with TTL and
duplicate suppression (``grpc_server.py:130-166``); non-direct peers are
reachable with ``create_connection`` (``grpc_client.py:142-144``) -- here every
peer of the machine is reachable on the bus.

A job (:class:`XgmiJob`) groups the peers that share a data plane: one rank
per process, a ``torch.distributed`` c10d store for rendezvous, the device.
``Node(..., protocol=job.protocol)`` creates the transport.
"""

from __future__ import annotations

import itertools
import os
import threading
import time
import uuid
from typing import Any, Callable, Dict, List, Optional

import msgpack
import torch

from p2pfl_amd.commands.command import Command
from p2pfl_amd.communication.client import BaseClient
from p2pfl_amd.communication.messages import Message, WeightsMessage
from p2pfl_amd.communication.neighbors import NeighborEntry, Neighbors
from p2pfl_amd.communication.protocol import BaseCommunicationProtocol
from p2pfl_amd.communication.server import ServerCore
from p2pfl_amd.communication.xgmi.bus import BusEndpoint
from p2pfl_amd.communication.xgmi.data_plane import SimFabric, XgmiDataPlane, make_backend_factory
from p2pfl_amd.learning.arena import FlatParams, ParamLayout
from p2pfl_amd.management.logger import logger
from p2pfl_amd.settings import Settings
from p2pfl_amd.utils.lockcheck import make_lock


def _pack(obj: Any) -> bytes:
    return msgpack.packb(obj, use_bin_type=True)


def _unpack(data: bytes) -> Any:
    return msgpack.unpackb(data, raw=False)


# ----------------------------------------------------------------------------
# job: the peers sharing one data plane
# ----------------------------------------------------------------------------
class XgmiJob:
    """Rank/world/store/device of this process's peer, and its data plane.

    ``backend``: ``"rccl"`` (GPU), ``"gloo"`` (CPU, multi-process),
    ``"sim"`` (in-process tests, needs ``fabric``), or ``"auto"``.
    :attr:`backend_in_use` is what the data plane actually agreed on.
    """

    def __init__(
        self,
        rank: int,
        world: int,
        store: Any,
        device: Optional[torch.device] = None,
        backend: str = "auto",
        prefix: str = "p2pfl",
        job_id: Optional[str] = None,
        fabric: Optional[SimFabric] = None,
        ack_timeout: float = 10.0,
        group_timeout: float = 60.0,
        rebuild_grace: float = 0.5,
        allow_fallback: bool = True,
    ) -> None:
        self.rank, self.world, self.store = rank, world, store
        # with the rccl backend: may the plane degrade to gloo through host
        # memory when RCCL cannot come up on every rank?  (False: the plane
        # fails and says why -- benchmarks must not report a gloo number as xGMI)
        self.allow_fallback = allow_fallback
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        if backend == "auto":
            from p2pfl_amd import ops

            backend = "rccl" if (self.device.type == "cuda" and ops.available()) else "gloo"
        self.backend = backend
        self.prefix = prefix
        self.job_id = job_id or os.environ.get("P2PFL_JOB_ID") or "job"
        self.fabric = fabric
        self.ack_timeout, self.group_timeout, self.rebuild_grace = ack_timeout, group_timeout, rebuild_grace
        self.plane: Optional[XgmiDataPlane] = None
        self._addr_cache: Dict[int, str] = {}
        self._rank_cache: Dict[str, int] = {}
        self._lock = make_lock("XgmiJob._lock")

    # -- addressing --------------------------------------------------------
    def address(self) -> str:
        return f"xgmi-{self.job_id}-{self.rank}"

    def protocol(self, addr: Optional[str] = None, commands: Optional[List[Command]] = None) -> "XgmiCommunicationProtocol":
        """Factory usable as ``Node(..., protocol=job.protocol)``."""
        if addr in (None, "", "127.0.0.1"):
            addr = self.address()
        return XgmiCommunicationProtocol(addr, commands, job=self)

    def publish(self, addr: str) -> None:
        self.store.set(f"{self.prefix}/addr/{self.rank}", addr)
        with self._lock:
            self._addr_cache[self.rank] = addr
            self._rank_cache[addr] = self.rank

    def rank_of(self, addr: str) -> Optional[int]:
        with self._lock:
            r = self._rank_cache.get(addr)
        if r is not None:
            return r
        for r in range(self.world):
            key = f"{self.prefix}/addr/{r}"
            with self._lock:
                if r in self._addr_cache:
                    continue
            if self.store.check([key]):
                a = self.store.get(key)
                a = a.decode() if isinstance(a, (bytes, bytearray)) else a
                with self._lock:
                    self._addr_cache[r] = a
                    self._rank_cache[a] = r
        with self._lock:
            return self._rank_cache.get(addr)

    # -- data plane ----------------------------------------------------------
    def start_plane(self, name: str) -> XgmiDataPlane:
        with self._lock:
            if self.plane is not None:
                return self.plane
            factory = make_backend_factory(
                self.backend, self.rank, self.store, f"{self.prefix}/plane", self.device, self.fabric, self.group_timeout
            )
            self.plane = XgmiDataPlane(
                self.rank, self.world, factory, store=self.store, prefix=f"{self.prefix}/plane", device=self.device,
                ack_timeout=self.ack_timeout, group_timeout=self.group_timeout, rebuild_grace=self.rebuild_grace,
                name=name, preconnect=self.backend == "rccl",
            )
            self.plane.allow_fallback = self.allow_fallback
            if self.backend == "rccl":
                # gloo staged through host memory if RCCL cannot come up on every rank
                self.plane.fallback = make_backend_factory(
                    "gloo", self.rank, self.store, f"{self.prefix}/plane", self.device, None, self.group_timeout
                )
            plane = self.plane
        plane.start()
        return plane

    @property
    def backend_in_use(self) -> Optional[str]:
        """The data plane's agreed backend once it is up (``None`` before / if it failed)."""
        plane = self.plane
        return plane.backend_name if plane is not None else None

    def stop_plane(self) -> None:
        with self._lock:
            plane, self.plane = self.plane, None
        if plane is not None:
            plane.stop()


class XgmiSimNetwork:
    """In-process peers on a simulated data plane (tests, examples without GPUs).

    ``net.protocol`` is a protocol *factory*: each call makes the next rank's
    transport, so ``Node(..., protocol=net.protocol)`` works like passing a
    protocol class.
    """

    def __init__(self, max_peers: int = 64, device: Optional[torch.device] = None) -> None:
        import torch.distributed as dist

        self.name = uuid.uuid4().hex[:8]
        self.store = dist.HashStore()
        self.fabric = SimFabric()
        self.max_peers = max_peers
        self.device = device
        self._ranks = itertools.count()
        self.jobs: List[XgmiJob] = []

    def protocol(self, addr: Optional[str] = None, commands: Optional[List[Command]] = None) -> "XgmiCommunicationProtocol":
        rank = next(self._ranks)
        if rank >= self.max_peers:
            raise RuntimeError("XgmiSimNetwork: too many peers")
        job = XgmiJob(rank, self.max_peers, self.store, device=self.device, backend="sim", job_id=self.name,
                      fabric=self.fabric, ack_timeout=2.0, group_timeout=10.0, rebuild_grace=0.2)
        self.jobs.append(job)
        return job.protocol(addr, commands)


# ----------------------------------------------------------------------------
# neighbours / client / server
# ----------------------------------------------------------------------------
class XgmiNeighbors(Neighbors):
    proto: "XgmiCommunicationProtocol"

    def connect(self, addr: str, non_direct: bool = False, handshake_msg: bool = True) -> NeighborEntry:
        if non_direct:
            return NeighborEntry(None, None, time.time())
        if handshake_msg:
            err = self.proto.request(addr, "hs", [self.self_addr], timeout=Settings.GRPC_TIMEOUT)
            if err:
                raise ConnectionError(f"Cannot add a neighbor: {err}")
        elif not self.proto.bus.reachable(addr):
            raise ConnectionError(f"{addr} is not reachable")
        return NeighborEntry(None, addr, time.time())

    def disconnect(self, addr: str, disconnect_msg: bool = True) -> None:
        if disconnect_msg:
            try:
                self.proto.bus.send(addr, _pack(["dc", self.self_addr]))
            except Exception:
                pass


class XgmiClient(BaseClient):
    proto: "XgmiCommunicationProtocol"

    def _deliver(self, handle: Any, msg: Any) -> Optional[str]:
        bus = self.proto.bus
        if isinstance(msg, Message):
            bus.send(handle, _pack(["m", msg.source, msg.ttl, msg.hash, msg.cmd, list(msg.args), msg.round]))
            return None
        if isinstance(msg, WeightsMessage):
            if isinstance(msg.weights, FlatParams) and self.proto.push_weights(handle, msg):
                return None
            payload = msg.weights
            if not isinstance(payload, (bytes, bytearray)):
                from p2pfl_amd.learning.wire import encode_params

                payload = encode_params(payload)
            bus.send(handle, _pack(["w", msg.source, msg.round, bytes(payload), list(msg.contributors), msg.weight, msg.cmd]))
            return None
        raise TypeError("Message type not supported.")

    def _temporary_handle(self, addr: str) -> Any:
        # every peer of the machine is reachable on the bus
        return addr if self.proto.bus.reachable(addr) else None


class XgmiServer(ServerCore):
    proto: "XgmiCommunicationProtocol"

    def start(self, wait: bool = False) -> None:
        proto = self.proto
        proto.bus = BusEndpoint(self.addr, proto._on_record, proto._on_peer_closed)
        proto.bus.start()

    def stop(self) -> None:
        if self.proto.bus is not None:
            self.proto.bus.close()


# ----------------------------------------------------------------------------
# protocol
# ----------------------------------------------------------------------------
class XgmiCommunicationProtocol(BaseCommunicationProtocol):
    neighbors_cls = XgmiNeighbors
    client_cls = XgmiClient
    server_cls = XgmiServer

    def __init__(self, addr: str = "127.0.0.1", commands: Optional[List[Command]] = None, job: Optional[XgmiJob] = None) -> None:
        if job is None:
            raise ValueError("XgmiCommunicationProtocol needs an XgmiJob (use Node(..., protocol=job.protocol))")
        self.job = job
        super().__init__(addr, commands)
        self._neighbors.proto = self  # type: ignore[attr-defined]
        self._client.proto = self  # type: ignore[attr-defined]
        self._server.proto = self  # type: ignore[attr-defined]
        self.bus: BusEndpoint = None  # type: ignore[assignment]
        self.plane: Optional[XgmiDataPlane] = None
        self._req_lock = make_lock("XgmiProtocol._req_lock")
        self._requests: Dict[int, List[Any]] = {}
        self._req_ids = itertools.count(1)
        self._layouts: Dict[str, ParamLayout] = {}
        self._layout_json: Dict[int, str] = {}
        self._departed: set = set()
        self._inbound: set = set()
        # keys of models already received (an identical proposal arriving
        # between the transfer and the handler's bookkeeping is declined).  Keys
        # carry the experiment generation: a second experiment on the same node
        # restarts at round 0 with the same (round, command, contributors).
        self._received: set = set()
        self._exp_gen = 0

    def _resolve_address(self, addr: str) -> str:
        if addr in (None, "", "127.0.0.1"):
            return self.job.address()
        return addr

    # -- lifecycle -------------------------------------------------------
    def start(self) -> None:
        super().start()  # server (bus endpoint), heartbeater, gossiper
        self.job.publish(self.addr)
        self.plane = self.job.start_plane(self.addr)
        self.plane.on_rebuild = self._announce_rebuild

    def stop(self) -> None:
        plane, self.plane = self.plane, None
        if self.bus is not None and plane is not None:
            # orderly exit: members must not treat the closing connection as a crash
            for r in plane.members:
                a = self.job._addr_cache.get(r)
                if a is not None and a != self.addr:
                    try:
                        self.bus.send(a, _pack(["bye"]))
                    except Exception:
                        pass
        if plane is not None:
            self.job.stop_plane()
        super().stop()

    @property
    def supports_device_payloads(self) -> bool:
        return True

    def experiment_boundary(self) -> None:
        """An experiment starts or ends on this node: forget the dedupe keys of the
        previous one (transfers still in flight finish under their old generation)."""
        with self._req_lock:
            self._exp_gen += 1
            self._received = set()
            self._inbound = set()

    # -- request / reply (handshake) ---------------------------------------
    def request(self, dst: str, kind: str, args: List[Any], timeout: float) -> Optional[str]:
        rid = next(self._req_ids)
        ev = threading.Event()
        slot: List[Any] = [ev, None]
        with self._req_lock:
            self._requests[rid] = slot
        try:
            self.bus.send(dst, _pack([kind, rid] + list(args)))
            if not ev.wait(timeout):
                return "timeout"
            return slot[1]
        finally:
            with self._req_lock:
                self._requests.pop(rid, None)

    def _reply(self, rid: int, err: Optional[str]) -> None:
        with self._req_lock:
            slot = self._requests.get(rid)
        if slot is not None:
            slot[1] = err
            slot[0].set()

    # -- weights over the data plane ------------------------------------------
    def _layout_str(self, layout: ParamLayout) -> str:
        key = id(layout)
        s = self._layout_json.get(key)
        if s is None:
            import json

            s = self._layout_json[key] = json.dumps(layout.to_json(), separators=(",", ":"))
        return s

    def push_weights(self, dst: str, msg: WeightsMessage) -> bool:
        """Send a device arena over the data plane; False if the plane cannot carry it."""
        plane = self.plane
        rank = self.job.rank_of(dst)
        if plane is None or rank is None or not plane.is_member(rank):
            return False
        if not plane.ready.wait(Settings.GRPC_TIMEOUT) or not plane.usable:
            return False
        params: FlatParams = msg.weights
        flat = params.flat
        if flat.device != plane.device:
            flat = flat.to(plane.device)
        if Settings.WIRE_DTYPE == "bf16" and flat.dtype == torch.float32:
            flat = flat.to(torch.bfloat16)
        nbytes = flat.numel() * flat.element_size()
        t_prop = time.perf_counter()

        feedback = msg.on_result

        def on_done(ok: bool, reason: str, evict: bool) -> None:
            if feedback is not None:
                try:
                    feedback("delivered" if ok else f"declined: {reason}")
                except Exception:
                    pass
            if ok:
                logger.tracer.count(self.addr, "xgmi_bytes_sent", nbytes)
                logger.tracer.count(self.addr, "xgmi_pushes")
                logger.tracer.record(self.addr, "xgmi_push", t_prop, time.perf_counter() - t_prop, to=dst, nbytes=nbytes)
                return
            logger.debug(self.addr, f"push of {msg.cmd} to {dst} not delivered: {reason}")
            if evict:
                logger.info(self.addr, f"push of {msg.cmd} to {dst} failed ({reason}); dropping the neighbour")
                self._neighbors.remove(dst)

        if feedback is not None:
            feedback("pending")
        hdr = plane.propose(rank, flat, on_done)
        hdr["rk"] = self.job.rank
        rec = ["wput", hdr, msg.source, msg.round, list(msg.contributors), msg.weight, msg.cmd,
               self._layout_str(params.layout)]
        try:
            self.bus.send(dst, _pack(rec))
        except Exception:
            plane.cancel(hdr["seq"], "header not delivered")
            if feedback is not None:
                feedback("declined: header not delivered")
            raise
        return True

    def _on_wput(self, src: str, rec: List[Any]) -> None:
        _, hdr, source, rnd, contributors, weight, cmd_name, layout_s = rec
        seq = hdr["seq"]

        def nack(reason: str, evict: bool) -> None:
            try:
                self.bus.send(src, _pack(["wnack", seq, reason, evict]))
            except Exception:
                pass

        cmd = self._server.commands.get(cmd_name)
        if cmd is None:
            logger.error(self.addr, f"Unknown command: {cmd_name} from {source}")
            return nack(f"Unknown command: {cmd_name}", True)
        pre = getattr(cmd, "precheck", None)
        if pre is not None:
            reason = pre(source, rnd, list(contributors), weight)
            if reason:
                logger.tracer.count(self.addr, "xgmi_pushes_declined")
                return nack(reason, False)
        plane = self.plane
        if plane is None or not plane.usable:
            return nack("data plane not running", False)
        # the same model already on its way here -- a re-send that crossed the
        # receiver's models_aggregated report, or the same contributor set from
        # another peer (an init model or a full aggregate offered by several
        # neighbours at once; equal contributors = the same average): one
        # transfer is enough
        with self._req_lock:
            gen = self._exp_gen
            key = (gen, rnd, cmd_name, tuple(sorted(contributors)))
            if key in self._inbound:
                return nack("already in flight", False)
            if key in self._received:
                return nack("already received", False)
            self._inbound.add(key)
        layout = self._layouts.get(layout_s)
        if layout is None:
            import json

            layout = self._layouts[layout_s] = ParamLayout.from_json(json.loads(layout_s))
        dev = plane.device

        def on_recv(buf: Optional[torch.Tensor], reason: str) -> None:
            with self._req_lock:
                self._inbound.discard(key)
                if buf is not None:
                    if len(self._received) > 4096:  # keep this experiment's recent rounds only
                        self._received = {k for k in self._received if k[0] == self._exp_gen and k[1] >= rnd - 2}
                    self._received.add(key)
            if buf is None:
                return
            if buf.is_cuda:
                # consumers run on the default stream: the buffer's block may
                # only be reused after their reads
                buf.record_stream(torch.cuda.default_stream(dev))
            logger.tracer.count(self.addr, "xgmi_bytes_recv", buf.numel() * buf.element_size())
            params = FlatParams.from_flat(buf, layout)
            err = self._server.handle_weights(WeightsMessage(source, rnd, params, list(contributors), weight, cmd_name))
            if err:
                try:
                    self.bus.send(src, _pack(["nack", cmd_name, err]))
                except Exception:
                    pass

        epoch, reason = plane.accept(int(hdr["rk"]), hdr, on_recv)
        if epoch is None:
            with self._req_lock:
                self._inbound.discard(key)
            return nack(reason, False)
        try:
            self.bus.send(src, _pack(["wack", seq, epoch, hdr["gen"]]))
        except Exception:
            pass

    def _announce_rebuild(self, gen: int) -> None:
        plane = self.plane
        if plane is None:
            return
        for r in plane.members:
            if r == self.job.rank:
                continue
            a = self.job._addr_cache.get(r)
            if a is None:
                continue
            try:
                self.bus.send(a, _pack(["prb", gen]))
            except Exception:
                pass

    # -- inbound records ------------------------------------------------------
    def _on_record(self, src: str, data: bytes) -> None:
        rec = _unpack(data)
        kind = rec[0]
        server = self._server
        if kind == "m":
            msg = Message(source=rec[1], ttl=rec[2], hash=rec[3], cmd=rec[4], args=list(rec[5]), round=rec[6])
            err = server.handle_message(msg)
            if err:
                try:
                    self.bus.send(src, _pack(["nack", msg.cmd, err]))
                except Exception:
                    pass
        elif kind == "nack":
            # an error reply drops the link on the sender's side (reference quirk Q13)
            logger.error(self.addr, f"Error while sending a message: {rec[1]}: {rec[2]}")
            self._neighbors.remove(src, disconnect_msg=True)
        elif kind == "hs":
            err = server.handle_handshake(rec[2])
            try:
                self.bus.send(src, _pack(["hsr", rec[1], err]))
            except Exception:
                pass
        elif kind == "hsr":
            self._reply(rec[1], rec[2])
        elif kind == "dc":
            server.handle_disconnect(rec[1])
        elif kind == "wput":
            self._on_wput(src, rec)
        elif kind == "wack":
            if self.plane is not None:
                self.plane.on_ack(rec[1], rec[2], rec[3])
        elif kind == "wnack":
            if self.plane is not None:
                self.plane.on_nack(rec[1], rec[2], bool(rec[3]))
        elif kind == "w":
            msg = WeightsMessage(rec[1], rec[2], rec[3], list(rec[4]), rec[5], rec[6])
            err = server.handle_weights(msg)
            if err:
                try:
                    self.bus.send(src, _pack(["nack", msg.cmd, err]))
                except Exception:
                    pass
        elif kind == "prb":
            if self.plane is not None:
                self.plane.request_rebuild(f"rebuild requested by {src}", gen=int(rec[1]))
        elif kind == "bye":
            self._departed.add(src)
        else:
            logger.error(self.addr, f"unknown control record {kind!r} from {src}")

    def _on_peer_closed(self, src: str) -> None:
        """The peer's process closed its connection: drop it now (no heartbeat wait)."""
        logger.info(self.addr, f"control connection from {src} closed")
        self._neighbors.remove(src, disconnect_msg=False)
        plane = self.plane
        if plane is not None and src not in self._departed:
            r = self.job.rank_of(src)
            if r is not None:
                plane.peer_lost(r)
