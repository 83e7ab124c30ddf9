"""Host control bus between the peers of one machine (the xGMI transport's C-plane).

Every peer process listens on an abstract-namespace ``AF_UNIX``
``SOCK_SEQPACKET`` socket named after its node address.  A send opens (once,
then caches) a connection to the destination and writes one record; records
keep their boundaries, are delivered in order per connection, and need no
framing, no TCP stack and no gRPC thread pool (the reference runs every control
message through a unary gRPC call and a 2-worker server pool:
``grpc_client.py:118-183``, ``grpc_server.py:62``).  Abstract sockets leave no
file behind when a process dies, and a dead peer is visible at once:

* a send to a peer whose process is gone fails with ``ECONNREFUSED`` /
  ``EPIPE`` -> ``ConnectionError`` (the client then drops the neighbour, as the
  reference does on any failed RPC);
* the receive side sees end-of-stream on the peer's connection and reports the
  peer through ``on_peer_closed`` (fast failure detection, ahead of the
  heartbeat timeout).

One dispatcher thread per endpoint multiplexes every inbound connection with
``selectors`` and hands each record to ``on_record``; handlers must not block
for long.  Weights normally never travel here, only their headers; when the
data plane cannot carry a model (it failed, or this rank was left out of a
rebuilt generation) the model goes out as one bus record anyway.  Records
larger than one socket packet (``MAX_RECORD``) are split into fragments that
are written back to back under the connection's lock and reassembled by the
receiver, so a 26 MB CNN or a 350 MB ViT still arrives -- slowly, through
host memory, but intact.
"""

from __future__ import annotations

import errno
import selectors
import socket
import threading
from typing import Callable, Dict, List, Optional

from p2pfl_amd.management.logger import logger
from p2pfl_amd.utils.lockcheck import make_lock

MAX_RECORD = 1 << 20
_HELLO = b"\x00P2FBUS1"
_HELLO_BULK = b"\x00P2FBULK"  # large-record connection (its close is not a peer exit)
# fragment of a large record: marker + 1 flag byte (1 = last fragment) + data
_FRAG = b"\x00P2FFRG"
FRAG_DATA = MAX_RECORD - len(_FRAG) - 1
MAX_MESSAGE = 2 << 30  # reassembly bound per record
SOCK_BUF = 4 << 20


def bus_name(addr: str) -> bytes:
    """Abstract-namespace socket name of a node address (<= 107 bytes)."""
    raw = ("p2pfl:" + addr).encode()
    if len(raw) > 107:
        import hashlib

        raw = b"p2pfl#" + hashlib.sha1(raw).hexdigest().encode()
    return b"\0" + raw


class BusEndpoint:
    """Listening endpoint + cached outbound connections of one node."""

    def __init__(
        self,
        addr: str,
        on_record: Callable[[str, bytes], None],
        on_peer_closed: Optional[Callable[[str], None]] = None,
    ) -> None:
        self.addr = addr
        self._on_record = on_record
        self._on_peer_closed = on_peer_closed
        self._lsock = socket.socket(socket.AF_UNIX, socket.SOCK_SEQPACKET)
        try:
            self._lsock.bind(bus_name(addr))
        except OSError as e:
            self._lsock.close()
            if e.errno == errno.EADDRINUSE:
                raise OSError(f"address {addr!r} is already used by another node on this machine") from e
            raise
        self._lsock.listen(512)
        self._lsock.setblocking(False)
        self._sel = selectors.DefaultSelector()
        self._sel.register(self._lsock, selectors.EVENT_READ, None)
        # wake-up pipe so close() interrupts select()
        self._wr, self._ww = socket.socketpair()
        self._wr.setblocking(False)
        self._sel.register(self._wr, selectors.EVENT_READ, "wake")
        self._out: Dict[tuple, socket.socket] = {}
        self._out_locks: Dict[tuple, threading.Lock] = {}
        self._out_lock = make_lock("BusEndpoint._out_lock")
        # inbound fragments of a large record, per connection (dispatcher thread only)
        self._partial: Dict[socket.socket, List[bytes]] = {}
        self._bulk: set = set()
        self._closed = threading.Event()
        self._thread = threading.Thread(target=self._loop, name=f"bus-{addr}", daemon=True)

    # ------------------------------------------------------------------
    def start(self) -> None:
        self._thread.start()

    def close(self) -> None:
        if self._closed.is_set():
            return
        self._closed.set()
        try:
            self._ww.send(b"x")
        except OSError:
            pass
        if self._thread.is_alive() and threading.current_thread() is not self._thread:
            self._thread.join(5)
        with self._out_lock:
            outs = list(self._out.values())
            self._out.clear()
        for s in outs:
            try:
                s.close()
            except OSError:
                pass
        for s in (self._lsock, self._wr, self._ww):
            try:
                s.close()
            except OSError:
                pass

    @property
    def closed(self) -> bool:
        return self._closed.is_set()

    # ------------------------------------------------------------------
    # send
    # ------------------------------------------------------------------
    def _connection(self, dst: str, bulk: bool = False) -> "tuple[socket.socket, threading.Lock]":
        key = (dst, bulk)
        with self._out_lock:
            s = self._out.get(key)
            if s is not None:
                return s, self._out_locks[key]
            lk = self._out_locks.get(key)
            if lk is None:
                lk = self._out_locks[key] = make_lock("BusEndpoint.conn_lock")
        # one connection per destination (plus one bulk connection for large
        # records): a second socket that said hello and then closed would look
        # like the peer's process going away
        with lk:
            with self._out_lock:
                s = self._out.get(key)
            if s is not None:
                return s, lk
            s = socket.socket(socket.AF_UNIX, socket.SOCK_SEQPACKET)
            try:
                s.setsockopt(socket.SOL_SOCKET, socket.SO_SNDBUF, SOCK_BUF)
                s.connect(bus_name(dst))
                s.sendall((_HELLO_BULK if bulk else _HELLO) + self.addr.encode())
            except OSError as e:
                s.close()
                raise ConnectionError(f"cannot reach {dst}: {e}") from e
            with self._out_lock:
                self._out[key] = s
            return s, lk

    def drop(self, dst: str, only_bulk: bool = False) -> None:
        """Forget the cached connections to ``dst`` (they will be reopened on demand).

        ``only_bulk``: drop just the bulk connection -- a failed large send must
        not close the control connection, whose close the peer reads as this
        node leaving."""
        with self._out_lock:
            socks = [self._out.pop((dst, b), None) for b in ((True,) if only_bulk else (False, True))]
        for s in socks:
            if s is not None:
                try:
                    s.close()
                except OSError:
                    pass

    def send(self, dst: str, record: bytes) -> None:
        if self._closed.is_set():
            raise ConnectionError("bus endpoint closed")
        if len(record) > MAX_MESSAGE:
            raise ValueError(f"bus record of {len(record)} bytes exceeds {MAX_MESSAGE}")
        # large records travel on their own connection, so control records
        # (acks, votes, heartbeats) never queue behind a multi-MB model and the
        # receiver's dispatcher never waits on a sender that waits on it
        bulk = len(record) > MAX_RECORD or record.startswith(_FRAG)
        s, lk = self._connection(dst, bulk)
        try:
            with lk:
                if not bulk:
                    s.sendall(record)
                else:
                    # fragments of one record are contiguous on the connection
                    # (the lock is held across all of them), so the receiver
                    # needs no record ids
                    view = memoryview(record)
                    for off in range(0, len(record), FRAG_DATA):
                        last = off + FRAG_DATA >= len(record)
                        s.sendall(_FRAG + (b"\x01" if last else b"\x00") + view[off : off + FRAG_DATA])
        except OSError as e:
            self.drop(dst, only_bulk=bulk)
            raise ConnectionError(f"send to {dst} failed: {e}") from e

    def reachable(self, dst: str) -> bool:
        try:
            self._connection(dst)
            return True
        except ConnectionError:
            return False

    # ------------------------------------------------------------------
    # receive
    # ------------------------------------------------------------------
    def _loop(self) -> None:
        peers: Dict[socket.socket, Optional[str]] = {}
        try:
            while not self._closed.is_set():
                for key, _ in self._sel.select(timeout=1.0):
                    sock = key.fileobj
                    if key.data == "wake":
                        return
                    if sock is self._lsock:
                        try:
                            conn, _ = self._lsock.accept()
                        except OSError:
                            continue
                        conn.setblocking(False)
                        conn.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, SOCK_BUF)
                        peers[conn] = None
                        self._sel.register(conn, selectors.EVENT_READ, "peer")
                        continue
                    self._drain(sock, peers)  # type: ignore[arg-type]
        except Exception as e:  # pragma: no cover - defensive
            if not self._closed.is_set():
                logger.error(self.addr, f"control bus loop died: {e}")
        finally:
            for s in list(peers):
                try:
                    self._sel.unregister(s)
                    s.close()
                except Exception:
                    pass
            try:
                self._sel.close()
            except Exception:
                pass

    def _drain(self, sock: socket.socket, peers: Dict[socket.socket, Optional[str]]) -> None:
        while True:
            try:
                data = sock.recv(MAX_RECORD)
            except BlockingIOError:
                return
            except OSError:
                data = b""
            if not data:  # peer closed its end (node stopped or process died)
                src = peers.pop(sock, None)
                self._partial.pop(sock, None)
                if sock in self._bulk:  # only the main connection's end means the peer left
                    self._bulk.discard(sock)
                    src = None
                try:
                    self._sel.unregister(sock)
                except Exception:
                    pass
                sock.close()
                if src is not None and self._on_peer_closed is not None and not self._closed.is_set():
                    try:
                        self._on_peer_closed(src)
                    except Exception as e:
                        logger.debug(self.addr, f"peer-closed handler failed: {e}")
                return
            src = peers.get(sock)
            if src is None:
                if data.startswith(_HELLO):
                    peers[sock] = data[len(_HELLO):].decode()
                elif data.startswith(_HELLO_BULK):
                    peers[sock] = data[len(_HELLO_BULK):].decode()
                    self._bulk.add(sock)
                continue
            if data.startswith(_FRAG):
                parts = self._partial.setdefault(sock, [])
                parts.append(data[len(_FRAG) + 1 :])
                if data[len(_FRAG)] != 1:
                    if sum(len(p) for p in parts) > MAX_MESSAGE:
                        logger.error(self.addr, f"oversized fragmented record from {src}; dropped")
                        self._partial.pop(sock, None)
                    continue
                data = b"".join(self._partial.pop(sock))
            try:
                self._on_record(src, data)
            except Exception as e:
                logger.error(self.addr, f"control record from {src} failed: {e}")

