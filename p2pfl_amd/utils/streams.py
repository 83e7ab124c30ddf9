"""Private HIP streams for learners and graph captures.

``torch.cuda.Stream()`` takes streams from a fixed per-device pool (32 per
priority, handed out round robin), so once a process holds more than 32 of
them -- virtual peers each own a compute, a validation and a capture stream --
two learners can silently share one HIP stream.  An event one peer records on
the shared stream while the other captures a HIP graph on it becomes a node of
that capture and every later use of it fails (``hipErrorCapturedEvent``;
``tests/test_gpu_node.py::test_virtual_peers_on_gpu``).  :func:`private_stream`
creates a stream of its own through the extension; it lives until the process
exits.
"""

from __future__ import annotations

import threading

import torch


# Private streams live until the process exits: nothing destroys them.  Destroying a
# stream while PyTorch still knows its handle is unsafe -- the caching allocator keeps
# recorded stream uses of freed blocks, and a graph keeps the stream it was captured on
# -- and the suite's exit crashed in the finalizer pass (weakref._exitfunc, SIGSEGV)
# while a destroy-on-collect scheme was in place.  A process creates a bounded number
# (a few per learner); the HIP runtime releases them at exit.
_STREAMS: list = []
_LOCK = threading.Lock()


def private_stream(device: torch.device, priority: int = 0) -> torch.cuda.Stream:
    """A non-blocking HIP stream no other caller is handed (see module doc).
    ``priority`` > 0: the device's lowest queue priority (work that should fill
    the gaps of other streams, e.g. evaluation passes beside training), < 0 its
    highest, 0 the default."""
    from p2pfl_amd.learning.step_graph import GATE
    from p2pfl_amd.ops import ext

    device = torch.device(device)
    idx = device.index if device.index is not None else torch.cuda.current_device()
    # created under the shared device gate: never while another thread records a graph
    with GATE.shared():
        handle = int(ext().new_stream(idx, int(priority)))
    s = torch.cuda.ExternalStream(handle, device=torch.device("cuda", idx))
    with _LOCK:
        _STREAMS.append(s)
    return s
