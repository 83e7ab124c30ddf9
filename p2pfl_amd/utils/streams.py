"""Private HIP streams for learners and graph captures.

``torch.cuda.Stream()`` takes streams from a fixed per-device pool (32 per
priority, handed out round robin), so once a process holds more than 32 of
them -- virtual peers each own a compute, a validation and a capture stream --
two learners can silently share one HIP stream.  An event one peer records on
the shared stream while the other captures a HIP graph on it becomes a node of
that capture and every later use of it fails (``hipErrorCapturedEvent``;
``tests/test_gpu_node.py::test_virtual_peers_on_gpu``).  :func:`private_stream`
creates a stream of its own through the extension and destroys it when the
returned wrapper is collected.
"""

from __future__ import annotations

import threading
import weakref

import torch


# Streams are never created or destroyed while another thread records a HIP graph:
# a finalizer (which runs inside whatever thread's garbage collection happens to
# fire) only queues the handle, and creation drains the queue under the shared
# device gate, which a capture holds exclusively (learning/step_graph.py).
_PENDING: list = []
_PENDING_LOCK = threading.Lock()


def _destroy(handle: int) -> None:
    with _PENDING_LOCK:
        _PENDING.append(handle)


def _drain() -> None:
    with _PENDING_LOCK:
        handles = _PENDING[:]
        del _PENDING[:]
    if not handles:
        return
    from p2pfl_amd.ops import ext

    for h in handles:
        try:
            ext().destroy_stream(h)
        except Exception:
            pass


def private_stream(device: torch.device) -> torch.cuda.Stream:
    """A non-blocking HIP stream no other caller is handed (see module doc)."""
    from p2pfl_amd.learning.step_graph import GATE
    from p2pfl_amd.ops import ext

    device = torch.device(device)
    idx = device.index if device.index is not None else torch.cuda.current_device()
    with GATE.shared():
        _drain()
        handle = int(ext().new_stream(idx))
    s = torch.cuda.ExternalStream(handle, device=torch.device("cuda", idx))
    weakref.finalize(s, _destroy, handle)
    return s
