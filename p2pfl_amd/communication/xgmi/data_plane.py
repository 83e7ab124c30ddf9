"""xGMI data plane: epoch-ordered grouped point-to-point weight transfers.

The reference pushes every model as a pickled byte string inside a unary gRPC
call (``grpc_client.py:118-183``), one neighbour after the other
(``gossiper.py:228-239``).  Here a model push is a device-to-device transfer of
the flat parameter arena over RCCL on ONE world communicator per job
generation, and all transfers a rank takes part in at a given moment -- its
k-way fan-out and the pushes it receives -- are launched as one
``ncclGroupStart/End`` group on a dedicated comm stream, so they run
concurrently on k xGMI links.

Why epochs.  RCCL point-to-point needs a matching receive, and the groups of
one communicator execute in issue order on each rank's stream.  Two ranks that
push to each other at the same moment would each block their stream on a send
whose matching receive sits *behind* the other rank's own send -- a deadlock --
unless both transfers are in the same group on both ranks.  Gossip pushes are
unsolicited, so the two sides first agree on WHEN a transfer runs:

1. the sender proposes the transfer with the lowest epoch it has not issued
   yet (``wput`` header on the control bus);
2. the receiver assigns ``epoch = max(proposal, its own lowest open epoch)``,
   reserves a receive buffer for it and replies (``wack``);
3. each rank issues, strictly in increasing epoch order, one group per epoch
   with all of its agreed sends and receives of that epoch; a rank does not
   issue an epoch while one of its own proposals that could still land in it
   is unanswered.

Every send in rank A's epoch-e group therefore has its receive in rank B's
epoch-e group, and each rank's stream holds its groups in epoch order.  By
induction on e, all groups of epochs < e complete, so every epoch-e group finds
its counterparts running: no cycle of waits can form, whatever the gossip
pattern (property-tested against a strict simulation of RCCL's stream-ordered
matching, :class:`SimFabric`).

Failure handling.  No host thread ever blocks inside RCCL (the communicator is
non-blocking; completion is an event polled with the GIL released).  A
proposal without an answer (receiver gone) fails after ``ack_timeout`` and the
caller drops the neighbour, like a failed gRPC call in the reference
(``grpc_client.py:159-179``).  When a member is lost (its control connection
closed, or heartbeat eviction, ``heartbeater.py:92-101``) every survivor
aborts the communicator -- releasing transfers that would wait for the dead
rank forever -- agrees on the surviving membership through the job's c10d
store, and builds generation g+1 over the survivors.  In-flight transfers fail
without evicting anyone; gossip re-sends them because the receivers'
``models_aggregated`` state did not change.

Backends: ``rccl`` (native, ``csrc/rccl_plane.cpp``), ``gloo`` (CPU tensors,
multi-process tests on machines without GPUs) and ``sim`` (in-process, strict
RCCL matching semantics, used by the single-process test-suite).
"""

from __future__ import annotations

import collections
import datetime
import json
import threading
import time
from abc import ABC, abstractmethod
from dataclasses import dataclass, field
from typing import Any, Callable, Deque, Dict, List, Optional, Tuple

import torch

from p2pfl_amd.management.logger import logger
from p2pfl_amd.utils.lockcheck import make_condition, make_lock

SEND, RECV = 0, 1


@dataclass
class Transfer:
    """One side of a weight transfer."""

    kind: int  # SEND / RECV
    peer: int  # global rank of the other side
    seq: int  # sender-assigned sequence number (unique per sender)
    tensor: torch.Tensor
    on_done: Callable[..., None]
    event: Any = None  # producer event a send must wait for (GPU)
    proposal: int = 0
    epoch: int = -1
    t0: float = field(default_factory=time.monotonic)


# ----------------------------------------------------------------------------
# backends
# ----------------------------------------------------------------------------
class Backend(ABC):
    name = "?"

    @abstractmethod
    def issue(self, ops: List[Transfer], index_of: Dict[int, int]) -> Any: ...

    @abstractmethod
    def poll(self, handle: Any) -> bool:
        """True when the group finished; raises if it failed."""

    def wait(self, handle: Any, timeout: float) -> bool:
        end = time.monotonic() + timeout
        while True:
            if self.poll(handle):
                return True
            if time.monotonic() >= end:
                return False
            time.sleep(0.0002)

    def release(self, handle: Any) -> None:
        pass

    def abort(self) -> None:
        pass

    def close(self) -> None:
        pass


class RcclBackend(Backend):
    """One RCCL communicator (native ``RcclPlane``) on a dedicated high-priority stream."""

    name = "rccl"

    def __init__(self, uid: bytes, members: List[int], rank: int, device: torch.device, group_timeout: float,
                 init_timeout: float = 120.0) -> None:
        from p2pfl_amd import ops

        self.device = torch.device(device)
        self.plane = ops.ext().RcclPlane(uid, len(members), members.index(rank), int(self.device.index or 0), init_timeout)
        self.stream = torch.cuda.ExternalStream(self.plane.stream, device=self.device)
        self.group_timeout = group_timeout

    def issue(self, ops: List[Transfer], index_of: Dict[int, int]) -> Any:
        for op in ops:
            if op.event is not None:
                self.stream.wait_event(op.event)
        return self.plane.issue([(op.kind, index_of[op.peer], op.tensor) for op in ops], [], self.group_timeout)

    def poll(self, handle: Any) -> bool:
        return bool(self.plane.query(handle))

    def wait(self, handle: Any, timeout: float) -> bool:
        return bool(self.plane.wait(handle, timeout))

    def release(self, handle: Any) -> None:
        self.plane.release(handle)

    def abort(self) -> None:
        self.plane.abort()

    def close(self) -> None:
        self.plane.close(5.0)


class GlooBackend(Backend):
    """Host tensors over a ``ProcessGroupGloo`` built straight from the store (no world group)."""

    name = "gloo"

    def __init__(self, store: Any, prefix: str, members: List[int], rank: int, timeout: float) -> None:
        import torch.distributed as dist

        self.pg = dist.ProcessGroupGloo(
            dist.PrefixStore(prefix, store), members.index(rank), len(members), datetime.timedelta(seconds=timeout)
        )

    def issue(self, ops: List[Transfer], index_of: Dict[int, int]) -> Any:
        works, stage = [], []
        for op in ops:
            t = op.tensor
            host = t if t.device.type == "cpu" else (t.cpu() if op.kind == SEND else torch.empty(t.shape, dtype=t.dtype))
            tag = op.epoch % (1 << 30)
            peer = index_of[op.peer]
            works.append(self.pg.send([host], peer, tag) if op.kind == SEND else self.pg.recv([host], peer, tag))
            if op.kind == RECV and host is not t:
                stage.append((host, t))
        return (works, stage)

    def poll(self, handle: Any) -> bool:
        works, _ = handle
        if not all(w.is_completed() for w in works):
            return False
        return self._finish(handle)

    def wait(self, handle: Any, timeout: float) -> bool:
        # gloo point-to-point works only complete inside wait() (is_completed()
        # stays False until then) and a second wait() on a finished receive
        # blocks for the next message: wait exactly once per work, from the
        # completer thread, bounded by the process group's own timeout
        works, _ = handle
        for w in works:
            w.wait()
        return self._finish(handle)

    @staticmethod
    def _finish(handle: Any) -> bool:
        _, stage = handle
        for host, dev in stage:
            dev.copy_(host)
        stage.clear()
        return True


class _SimGroup:
    def __init__(self, rank: int, ops: List[Tuple[int, int, torch.Tensor]]) -> None:
        self.rank = rank
        self.ops = ops
        self.matched = [False] * len(ops)
        self.done = threading.Event()
        self.error: Optional[str] = None


class SimFabric:
    """In-process model of RCCL point-to-point semantics, for tests.

    Each rank has a stream of groups that run strictly in issue order; a
    group's send to B can only be matched by a receive from A in B's *running*
    (oldest unfinished) group, in per-pair FIFO order; a group finishes when
    all its operations are matched.  A schedule that would deadlock on RCCL
    never finishes here either.
    """

    _registry: Dict[str, "SimFabric"] = {}
    _reg_lock = threading.Lock()

    def __init__(self) -> None:
        self._lock = threading.Lock()
        self._streams: Dict[int, Deque[_SimGroup]] = collections.defaultdict(collections.deque)
        self._dead: set = set()

    @classmethod
    def get(cls, name: str) -> "SimFabric":
        with cls._reg_lock:
            f = cls._registry.get(name)
            if f is None:
                f = cls._registry[name] = SimFabric()
            return f

    @classmethod
    def drop(cls, name: str) -> None:
        with cls._reg_lock:
            cls._registry.pop(name, None)

    def issue(self, rank: int, ops: List[Tuple[int, int, torch.Tensor]]) -> _SimGroup:
        g = _SimGroup(rank, ops)
        with self._lock:
            if rank in self._dead:
                g.error = "rank is dead"
                g.done.set()
                return g
            self._streams[rank].append(g)
            self._progress()
        return g

    def kill(self, rank: int) -> None:
        """Simulate a crashed rank: its queued groups never run."""
        with self._lock:
            self._dead.add(rank)

    def abort(self, rank: int) -> None:
        with self._lock:
            for g in self._streams.pop(rank, ()):
                g.error = "aborted"
                g.done.set()

    def _progress(self) -> None:
        changed = True
        while changed:
            changed = False
            for rank, q in list(self._streams.items()):
                if not q or rank in self._dead:
                    continue
                g = q[0]
                for i, (kind, peer, t) in enumerate(g.ops):
                    if g.matched[i] or kind != SEND:
                        continue
                    pq = self._streams.get(peer)
                    if not pq or peer in self._dead:
                        continue
                    pg = pq[0]
                    # first unmatched receive from `rank` in the peer's running group
                    for j, (k2, p2, t2) in enumerate(pg.ops):
                        if k2 == RECV and p2 == rank and not pg.matched[j]:
                            # FIFO per pair: all earlier sends rank->peer in g must be matched already
                            if any(not g.matched[x] and g.ops[x][0] == SEND and g.ops[x][1] == peer for x in range(i)):
                                break
                            if t2.numel() * t2.element_size() != t.numel() * t.element_size():
                                g.error = pg.error = "size mismatch"
                            else:
                                t2.view(-1).view(torch.uint8).copy_(t.reshape(-1).view(torch.uint8))
                            g.matched[i] = pg.matched[j] = True
                            changed = True
                            break
                for r2, q2 in list(self._streams.items()):
                    while q2 and all(q2[0].matched):
                        q2.popleft().done.set()
                        changed = True


class SimBackend(Backend):
    name = "sim"

    def __init__(self, fabric: SimFabric, members: List[int], rank: int) -> None:
        self.fabric = fabric
        self.rank = rank

    def issue(self, ops: List[Transfer], index_of: Dict[int, int]) -> Any:
        return self.fabric.issue(self.rank, [(op.kind, op.peer, op.tensor) for op in ops])

    def poll(self, handle: Any) -> bool:
        if not handle.done.is_set():
            return False
        if handle.error:
            raise RuntimeError(f"sim transfer failed: {handle.error}")
        return True

    def wait(self, handle: Any, timeout: float) -> bool:
        handle.done.wait(timeout)
        return self.poll(handle)

    def abort(self) -> None:
        self.fabric.abort(self.rank)


# ----------------------------------------------------------------------------
# membership
# ----------------------------------------------------------------------------
def agree_members(store: Any, prefix: str, gen: int, rank: int, world: int, lost: List[int], grace: float,
                  wait_all: float = 5.0) -> List[int]:
    """Survivors of generation ``gen - 1`` agree on the members of generation ``gen``.

    Each survivor announces itself and waits until every rank it does not
    know to be lost has announced too (at most ``max(grace, wait_all)``
    seconds: a rank that died unnoticed is not waited for forever, and the
    common case needs no fixed sleep), then proposes the set of announced
    ranks; the first proposal stored wins (compare-and-set), so every survivor
    builds the communicator over the same list.  A survivor that announces too
    late to be included asks for generation ``gen + 1`` instead of giving up
    (:meth:`XgmiDataPlane._rebuild`).
    """
    base = f"{prefix}/g{gen}"
    store.set(f"{base}/alive/{rank}", "1")
    expect = [f"{base}/alive/{r}" for r in range(world) if r not in lost]
    t0 = time.monotonic()
    while True:
        if store.check([f"{base}/members"]):
            break  # someone already decided; joining late changes nothing
        if all(store.check([k]) for k in expect):
            break
        waited = time.monotonic() - t0
        if waited >= max(grace, wait_all):
            break
        time.sleep(0.005)
    # every announced rank is alive, including one the others had written off
    # (left out of an earlier generation): only ranks that never announce stay out
    alive = [r for r in range(world) if store.check([f"{base}/alive/{r}"])]
    if rank not in alive:
        alive.append(rank)
    got = store.compare_set(f"{base}/members", "", json.dumps(sorted(alive)))
    return list(json.loads(got.decode() if isinstance(got, (bytes, bytearray)) else got))


# ----------------------------------------------------------------------------
# the plane
# ----------------------------------------------------------------------------
class XgmiDataPlane:
    """Per-rank scheduler of epoch-grouped weight transfers (see module docstring)."""

    def __init__(
        self,
        rank: int,
        world: int,
        make_backend: Callable[[int, List[int]], Backend],
        store: Any = None,
        prefix: str = "p2pfl/plane",
        device: Optional[torch.device] = None,
        ack_timeout: float = 10.0,
        group_timeout: float = 60.0,
        rebuild_grace: float = 0.5,
        name: str = "",
        preconnect: bool = True,
    ) -> None:
        self.rank, self.world = rank, world
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self._make_backend = make_backend
        self._store = store
        self._prefix = prefix
        self.ack_timeout, self.group_timeout, self.rebuild_grace = ack_timeout, group_timeout, rebuild_grace
        self.name = name or f"rank{rank}"
        self.preconnect = preconnect
        self._cv = make_condition("XgmiDataPlane._cv")
        self.gen = 0
        self.members: List[int] = list(range(world))
        self._index = {r: i for i, r in enumerate(self.members)}
        self._lost: set = set()
        self._backend: Optional[Backend] = None
        self._seq = 0
        self._open = 0  # lowest epoch not issued yet
        self._pending: Dict[int, List[Transfer]] = collections.defaultdict(list)
        self._outstanding: Dict[int, Transfer] = {}  # my proposals awaiting an answer
        self._inflight: Deque[Tuple[Any, List[Transfer], float]] = collections.deque()
        self._stopped = False
        self._rebuilding = False
        self.ready = threading.Event()
        self.failed: Optional[str] = None
        self.stats = collections.Counter()
        # generation-0 backend actually in use ("rccl", or "gloo" after a fallback)
        self.backend_name: Optional[str] = None
        self.fallback_reason: Optional[str] = None
        # False: a failed primary backend fails the plane instead of degrading
        self.allow_fallback = True
        self._late_joins = 0
        self.max_late_joins = 3
        self._issuer = threading.Thread(target=self._issue_loop, name=f"xgmi-issue-{self.name}", daemon=True)
        self._completer = threading.Thread(target=self._complete_loop, name=f"xgmi-complete-{self.name}", daemon=True)
        self._alloc_stream: Any = None
        # set by the transport: tell the other members to join generation g
        self.on_rebuild: Optional[Callable[[int], None]] = None
        # generation-0 backend every rank switches to if the primary fails on any
        self.fallback: Optional[Callable[[int, List[int]], Backend]] = None

    # ------------------------------------------------------------------
    # lifecycle
    # ------------------------------------------------------------------
    def start(self, block: bool = False) -> None:
        """Build generation 0 (collective over all ranks) in the background."""
        t = threading.Thread(target=self._init, name=f"xgmi-init-{self.name}", daemon=True)
        t.start()
        if block:
            t.join()

    def _init(self) -> None:
        try:
            backend = self._agreed_backend()
            with self._cv:
                self._backend = backend
                self._alloc_stream = getattr(backend, "stream", None)
            self._issuer.start()
            self._completer.start()
            if self.preconnect:
                self._preconnect()
            self.ready.set()
        except Exception as e:
            self.failed = f"data plane init failed: {e}"
            logger.error(self.name, self.failed)
            self.ready.set()

    def _agreed_backend(self) -> Backend:
        """Generation 0's backend; with a fallback, every rank switches together.

        Each rank reports whether its primary backend (RCCL) came up; if any
        rank failed, all of them build the fallback (gloo through host memory)
        instead -- a federation that runs slower rather than one that cannot
        move models at all.
        """
        members = list(self.members)
        try:
            backend, err = self._make_backend(0, members), None
        except Exception as e:  # noqa: BLE001
            backend, err = None, e
        if self.fallback is None or self._store is None or self.world == 1:
            if backend is None:
                raise err  # type: ignore[misc]
            self.backend_name = backend.name
            return backend
        keys = [f"{self._prefix}/g0/ok/{r}" for r in members]
        self._store.set(keys[members.index(self.rank)], "1" if backend is not None else "0")
        self._store.wait(keys, datetime.timedelta(seconds=self.group_timeout * 2))
        if all(bytes(self._store.get(k)) == b"1" for k in keys):
            self.backend_name = backend.name  # type: ignore[union-attr]
            return backend  # type: ignore[return-value]
        failed_on = [r for r, k in zip(members, keys) if bytes(self._store.get(k)) != b"1"]
        self.fallback_reason = f"primary backend failed on rank(s) {failed_on}" + (f": {err}" if err else "")
        if backend is not None:
            try:
                backend.abort()
            except Exception:
                pass
        if not self.allow_fallback:
            raise RuntimeError(f"{self.fallback_reason}; fallback disallowed")
        logger.warning(self.name, f"xgmi data plane: {self.fallback_reason}; using the fallback")
        fb = self.fallback(0, members)
        self.backend_name = fb.name
        return fb

    def _preconnect(self) -> None:
        """Epoch 0: exchange one element with every member (opens every xGMI
        peer connection outside any timed region and proves the plane works)."""
        if len(self.members) < 2:
            return
        done = threading.Semaphore(0)
        n = 0
        with self._cv:
            for r in self.members:
                if r == self.rank:
                    continue
                for kind in (SEND, RECV):
                    t = self._alloc(1, torch.float32)
                    if kind == SEND:
                        t.fill_(float(self.rank))
                    op = Transfer(kind, r, -1, t, lambda *a, **k: done.release(), epoch=0)
                    self._pending[0].append(op)
                    n += 1
            self._cv.notify_all()
        for _ in range(n):
            if not done.acquire(timeout=self.group_timeout):
                raise TimeoutError("pre-connect exchange timed out")

    def stop(self) -> None:
        with self._cv:
            if self._stopped:
                return
            self._stopped = True
            self._cv.notify_all()
            backend = self._backend
        for th in (self._issuer, self._completer):
            if th.is_alive() and th is not threading.current_thread():
                th.join(5)
        self._fail_all("data plane stopped")
        if backend is not None:
            try:
                backend.close()
            except Exception:
                pass

    @property
    def usable(self) -> bool:
        return self.ready.is_set() and self.failed is None and not self._stopped

    def is_member(self, rank: int) -> bool:
        return rank in self._index and rank not in self._lost

    # ------------------------------------------------------------------
    # buffers
    # ------------------------------------------------------------------
    def _alloc(self, numel: int, dtype: torch.dtype) -> torch.Tensor:
        if self.device.type == "cuda" and self._alloc_stream is not None:
            # allocated in the comm stream's pool: reuse is ordered after the transfers
            with torch.cuda.stream(self._alloc_stream):
                return torch.empty(numel, dtype=dtype, device=self.device)
        return torch.empty(numel, dtype=dtype, device=self.device)

    # ------------------------------------------------------------------
    # sender side
    # ------------------------------------------------------------------
    def propose(self, dst: int, tensor: torch.Tensor, on_done: Callable[..., None]) -> Dict[str, Any]:
        """Register a push of ``tensor`` to rank ``dst``; returns the header fields to send.

        ``on_done(ok, reason, evict)`` runs once the transfer finished or failed.
        """
        if not self.is_member(dst):
            raise ConnectionError(f"rank {dst} is not a data-plane member")
        ev = None
        if tensor.is_cuda:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(tensor.device))
        with self._cv:
            if self._stopped or self.failed:
                raise ConnectionError(self.failed or "data plane stopped")
            self._seq += 1
            op = Transfer(SEND, dst, self._seq, tensor.reshape(-1), on_done, event=ev, proposal=self._open)
            self._outstanding[op.seq] = op
            self.stats["proposed"] += 1
            return {"seq": op.seq, "ep": op.proposal, "gen": self.gen, "n": int(op.tensor.numel()),
                    "dt": str(op.tensor.dtype).replace("torch.", "")}

    def cancel(self, seq: int, reason: str) -> None:
        """The header never reached the receiver: drop the proposal (no callback)."""
        with self._cv:
            self._outstanding.pop(seq, None)
            self._cv.notify_all()

    def on_ack(self, seq: int, epoch: int, gen: int) -> None:
        with self._cv:
            op = self._outstanding.pop(seq, None)
            if op is None:
                return
            bad = None
            if gen != self.gen:
                bad = "stale data-plane generation"
            elif int(epoch) < self._open:  # impossible: an unanswered proposal blocks its epoch
                bad = f"acknowledged into issued epoch {epoch} < {self._open}"
            else:
                op.epoch = int(epoch)
                self._pending[op.epoch].append(op)
            self._cv.notify_all()
        if bad is None:
            logger.tracer.record(self.name, "xgmi_ack", op.t0, time.monotonic() - op.t0, peer=op.peer, epoch=op.epoch)
        if bad is not None:
            logger.error(self.name, f"xgmi push {seq} dropped: {bad}")
            self._done(op, False, bad, False)

    def on_nack(self, seq: int, reason: str, evict: bool) -> None:
        with self._cv:
            op = self._outstanding.pop(seq, None)
            self._cv.notify_all()
        if op is not None:
            self.stats["nacked"] += 1
            # per-reason tally ("late round (3 != 2)" -> "late round")
            self.stats["nacked/" + reason.split(" (")[0]] += 1
            self._done(op, False, reason, evict)

    # ------------------------------------------------------------------
    # receiver side
    # ------------------------------------------------------------------
    def accept(self, src: int, hdr: Dict[str, Any], on_recv: Callable[..., None]) -> Tuple[Optional[int], str]:
        """Reserve a receive for a proposal; returns (epoch, "") or (None, reason)."""
        if not self.is_member(src):
            return None, "sender is not a data-plane member"
        if int(hdr["gen"]) != self.gen:
            return None, "stale data-plane generation"
        dtype = getattr(torch, str(hdr["dt"]))
        buf = self._alloc(int(hdr["n"]), dtype)
        with self._cv:
            if self._stopped or self._rebuilding or self.failed:
                return None, "data plane not running"
            if int(hdr["gen"]) != self.gen:
                return None, "stale data-plane generation"
            e = max(int(hdr["ep"]), self._open)
            op = Transfer(RECV, src, int(hdr["seq"]), buf, on_recv, epoch=e)
            self._pending[e].append(op)
            self.stats["accepted"] += 1
            self._cv.notify_all()
        return e, ""

    # ------------------------------------------------------------------
    # issue / complete
    # ------------------------------------------------------------------
    def _issuable_locked(self) -> Optional[int]:
        if not self._pending or self._backend is None or self._rebuilding:
            return None
        e0 = min(self._pending)
        if any(op.proposal <= e0 for op in self._outstanding.values()):
            return None
        return e0

    def _issue_loop(self) -> None:
        while True:
            expired: List[Transfer] = []
            with self._cv:
                while not self._stopped:
                    now = time.monotonic()
                    expired = [op for op in self._outstanding.values() if now - op.t0 > self.ack_timeout]
                    for op in expired:
                        self._outstanding.pop(op.seq, None)
                    if expired or self._issuable_locked() is not None:
                        break
                    self._cv.wait(timeout=0.05)
                if self._stopped:
                    return
                e0 = self._issuable_locked()
                ops = self._pending.pop(e0) if e0 is not None else []
                if e0 is not None:
                    self._open = e0 + 1
                backend, index, gen = self._backend, dict(self._index), self.gen
            for op in expired:
                self.stats["ack_timeout"] += 1
                self._done(op, False, "no answer from the receiver", True)
            if not ops:
                continue
            t_issue = time.monotonic()
            try:
                h = backend.issue(ops, index)
            except Exception as e:
                logger.error(self.name, f"xgmi group (epoch {e0}) failed to launch: {e}")
                for op in ops:
                    self._done(op, False, f"launch failed: {e}", False)
                if gen == self.gen:
                    self.request_rebuild(f"launch failure: {e}")
                continue
            self.stats["groups"] += 1
            with self._cv:
                self._inflight.append((h, ops, t_issue, gen))
                self._cv.notify_all()

    def _complete_loop(self) -> None:
        while True:
            with self._cv:
                while not self._inflight and not self._stopped:
                    self._cv.wait(timeout=0.2)
                if self._stopped:
                    return
                h, ops, t0, gen = self._inflight[0]
                backend = self._backend
            try:
                done = backend.wait(h, 0.05)
            except Exception as e:
                with self._cv:
                    if self._inflight and self._inflight[0][0] is h:
                        self._inflight.popleft()
                logger.error(self.name, f"xgmi transfer failed: {e}")
                for op in ops:
                    self._done(op, False, f"transfer failed: {e}", False)
                if gen == self.gen and not self._rebuilding:  # not a casualty of our own abort
                    self.request_rebuild(f"transfer failure: {e}")
                continue
            if not done:
                if time.monotonic() - t0 > self.group_timeout and gen == self.gen and not self._rebuilding:
                    logger.error(self.name, f"xgmi group stuck for {self.group_timeout}s; rebuilding the communicator")
                    self.request_rebuild("group timeout")
                continue
            with self._cv:
                if self._inflight and self._inflight[0][0] is h:
                    self._inflight.popleft()
            try:
                backend.release(h)
            except Exception:
                pass
            t_done = time.monotonic()
            nbytes = sum(op.tensor.numel() * op.tensor.element_size() for op in ops)
            logger.tracer.record(self.name, "xgmi_group", t0, t_done - t0, epoch=ops[0].epoch, ops=len(ops), nbytes=nbytes)
            for op in ops:
                if op.seq >= 0:  # not the pre-connect exchange
                    key = "link_tx_bytes" if op.kind == SEND else "link_rx_bytes"
                    logger.tracer.count(self.name, f"{key}/{op.peer}", op.tensor.numel() * op.tensor.element_size())
            for op in ops:
                if op.kind == SEND:
                    self.stats["sent"] += 1
                    self.stats["bytes_sent"] += op.tensor.numel() * op.tensor.element_size()
                    self._done(op, True, "", False)
                else:
                    self.stats["received"] += 1
                    self.stats["bytes_recv"] += op.tensor.numel() * op.tensor.element_size()
                    self._done(op, True, "", False)

    def _done(self, op: Transfer, ok: bool, reason: str, evict: bool) -> None:
        try:
            if op.kind == SEND:
                op.on_done(ok, reason, evict)
            else:
                op.on_done(op.tensor if ok else None, reason)
        except Exception as e:
            logger.error(self.name, f"xgmi completion callback failed: {e}")

    def _fail_all(self, reason: str) -> None:
        with self._cv:
            ops = [op for entry in self._inflight for op in entry[1]]
            ops += [op for group in self._pending.values() for op in group]
            ops += list(self._outstanding.values())
            self._inflight.clear()
            self._pending.clear()
            self._outstanding.clear()
        for op in ops:
            self._done(op, False, reason, False)

    # ------------------------------------------------------------------
    # membership changes
    # ------------------------------------------------------------------
    def peer_lost(self, rank: int) -> None:
        """A member left (process gone, or an orderly exit).

        Work with it that was agreed but not launched is dropped; if a launched
        group still waits on it, the communicator is aborted and every survivor
        moves to a new generation (a launched RCCL transfer cannot be cancelled).
        """
        with self._cv:
            if rank not in self._index or rank in self._lost or rank == self.rank:
                return
            self._lost.add(rank)
            dropped = [op for op in self._outstanding.values() if op.peer == rank]
            for op in dropped:
                self._outstanding.pop(op.seq, None)
            for e in list(self._pending):
                keep = [op for op in self._pending[e] if op.peer != rank]
                dropped += [op for op in self._pending[e] if op.peer == rank]
                if keep:
                    self._pending[e] = keep
                else:
                    del self._pending[e]
            stuck = any(op.peer == rank for entry in self._inflight for op in entry[1])
            self._cv.notify_all()
        for op in dropped:
            self._done(op, False, f"rank {rank} left", False)
        if stuck:
            self.request_rebuild(f"rank {rank} lost with transfers in flight")

    def request_rebuild(self, reason: str, gen: Optional[int] = None) -> None:
        """Move to generation ``gen`` (default: the next one).  Peers are told
        through ``on_rebuild`` so that every survivor joins the agreement."""
        with self._cv:
            if self._stopped or self._store is None:
                return
            target = self.gen + 1 if gen is None else int(gen)
            if target <= self.gen and (self._rebuilding or gen is not None):
                return
            self._rebuilding = True
            self.gen = target
            backend = self._backend
        logger.info(self.name, f"xgmi data plane: {reason}; building generation {target}")
        if self.on_rebuild is not None:
            try:
                self.on_rebuild(target)
            except Exception:
                pass
        threading.Thread(target=self._rebuild, args=(target, backend), name=f"xgmi-rebuild-{self.name}", daemon=True).start()

    def _rebuild(self, gen: int, old: Optional[Backend]) -> None:
        if self._stopped:
            return
        if old is not None:
            try:
                old.abort()
            except Exception:
                pass
        self._fail_all("data plane rebuilding after a membership change")
        try:
            members = agree_members(self._store, self._prefix, gen, self.rank, self.world, sorted(self._lost), self.rebuild_grace)
            if self.rank not in members:
                # announced too late for generation `gen`: ask everyone to
                # build gen + 1 (which waits for this rank's announcement)
                # instead of failing for good
                self._late_joins += 1
                if self._late_joins <= self.max_late_joins:
                    logger.info(self.name, f"left out of data-plane generation {gen}; requesting generation {gen + 1}")
                    # announce for gen + 1 BEFORE asking for it: the others
                    # have written this rank off as lost and would not wait
                    self._store.set(f"{self._prefix}/g{gen + 1}/alive/{self.rank}", "1")
                    self.request_rebuild("rejoin after being left out", gen=gen + 1)
                    return
                raise RuntimeError("excluded from the new generation")
            if self._stopped:
                return
            backend = self._make_backend(gen, members)
        except Exception as e:
            with self._cv:
                if self.gen != gen:
                    return  # superseded by a newer generation while agreeing
                self.failed = f"data plane rebuild failed: {e}"
                self._rebuilding = False
                self._cv.notify_all()
            logger.error(self.name, self.failed)
            return
        with self._cv:
            superseded = self.gen != gen  # a newer generation was requested meanwhile
            if not superseded:
                self.members = members
                self._index = {r: i for i, r in enumerate(members)}
                self._lost = (self._lost | {r for r in range(self.world) if r not in members}) - set(members)
                self._backend = backend
                self.backend_name = getattr(backend, "name", self.backend_name)  # what generation `gen` runs on
                self._alloc_stream = getattr(backend, "stream", None)
                self._open = 0
                self._rebuilding = False
                self.stats["rebuilds"] += 1
                self._cv.notify_all()
        if superseded:
            try:
                backend.abort()
            except Exception:
                pass
            return
        logger.info(self.name, f"xgmi data plane generation {gen} up: members {members}")


def make_backend_factory(kind: str, rank: int, store: Any, prefix: str, device: torch.device,
                         fabric: Optional[SimFabric] = None, timeout: float = 60.0) -> Callable[[int, List[int]], Backend]:
    """Backend constructor for generation ``gen`` over ``members``."""

    def factory(gen: int, members: List[int]) -> Backend:
        base = f"{prefix}/g{gen}"
        if kind == "rccl":
            from p2pfl_amd import ops

            key = f"{base}/uid"
            if rank == members[0]:
                store.set(key, ops.ext().rccl_unique_id())
            uid = store.get(key)  # blocks until the first member published it
            return RcclBackend(bytes(uid), members, rank, device, timeout, init_timeout=max(timeout, 30.0))
        if kind == "gloo":
            return GlooBackend(store, base + "/gloo", members, rank, timeout)
        if kind == "sim":
            assert fabric is not None
            return SimBackend(fabric, members, rank)
        raise ValueError(f"unknown data-plane backend {kind!r}")

    return factory
