"""RCCL data plane on a real MI355X (one GPU: a 1-rank communicator, self send/recv).

The multi-rank schedule is covered on the CPU (strict simulator, gloo
processes); here the native ``RcclPlane`` binding and the epoch scheduler run
on the device: non-blocking communicator init from a store-exchanged unique
id, grouped send+recv on the dedicated comm stream, completion polling,
producer-event ordering, abort.
"""

from __future__ import annotations

import threading

import pytest
import torch

pytestmark = pytest.mark.gpu


def _plane():
    import torch.distributed as dist

    from p2pfl_amd.communication.xgmi.data_plane import XgmiDataPlane, make_backend_factory

    dev = torch.device("cuda", 0)
    store = dist.HashStore()
    plane = XgmiDataPlane(0, 1, make_backend_factory("rccl", 0, store, "t", dev), store=store, prefix="t", device=dev,
                          preconnect=False)
    plane.start(block=True)
    assert plane.failed is None, plane.failed
    return plane, dev


def _self_push(plane, t):
    got = {}
    done = threading.Event()

    def on_send(ok, reason, evict):
        got["send"] = (ok, reason)

    def on_recv(buf, reason):
        got["buf"] = buf
        done.set()

    hdr = plane.propose(0, t, on_send)
    e, why = plane.accept(0, hdr, on_recv)
    assert e is not None, why
    plane.on_ack(hdr["seq"], e, hdr["gen"])
    assert done.wait(30), "RCCL self transfer did not complete"
    return got


def test_rccl_plane_self_transfer_bitexact():
    from p2pfl_amd import ops

    ops.ext()
    plane, dev = _plane()
    try:
        # a CNN-sized arena (6.5 M fp32) produced by a kernel just before the push:
        # the comm stream must wait for it (producer event)
        n = 6_497_280
        src = torch.empty(n, device=dev)
        src.copy_(torch.randn(n, device=dev))
        got = _self_push(plane, src)
        assert got["send"] == (True, "")
        torch.testing.assert_close(got["buf"], src, rtol=0, atol=0)
        # bf16 arenas (opt-in wire dtype) move as raw bytes too
        h = torch.randn(4099, device=dev).to(torch.bfloat16)
        got = _self_push(plane, h)
        assert got["buf"].dtype == torch.bfloat16 and torch.equal(got["buf"], h)
        assert plane.stats["groups"] >= 2 and plane.stats["bytes_sent"] >= n * 4
    finally:
        plane.stop()


def test_rccl_plane_native_binding_checks_and_abort():
    from p2pfl_amd import ops

    C = ops.ext()
    p = C.RcclPlane(C.rccl_unique_id(), 1, 0, 0, 60.0)
    dev = torch.device("cuda", 0)
    a = torch.arange(1024, dtype=torch.float32, device=dev)
    b = torch.zeros_like(a)
    gid = p.issue([(0, 0, a), (1, 0, b)], [torch.cuda.current_stream(dev).cuda_stream], 30.0)
    assert p.wait(gid, 30.0) == 1
    p.release(gid)
    torch.testing.assert_close(a, b)
    with pytest.raises(RuntimeError):
        p.issue([(0, 3, a)], [], 5.0)  # peer out of range: refused on the host
    with pytest.raises(RuntimeError):
        p.issue([(0, 0, a.cpu())], [], 5.0)  # host tensor: refused on the host
    p.abort()
    assert p.aborted
    with pytest.raises(RuntimeError):
        p.issue([(0, 0, a)], [], 5.0)
