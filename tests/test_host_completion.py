"""HostCompletions: deferred host work of enqueued GPU passes runs in order, after its event."""

from __future__ import annotations

import threading
import time

from p2pfl_amd.learning.host_completion import HostCompletions


class _Ev:
    def __init__(self) -> None:
        self.fired = threading.Event()

    def synchronize(self) -> None:
        self.fired.wait()


def test_callbacks_run_after_their_event_in_fifo_order_and_drain_waits():
    hc = HostCompletions("t")
    out = []
    evs = [_Ev() for _ in range(3)]
    for i, ev in enumerate(evs):
        hc.submit(ev, lambda i=i: out.append(i))
    time.sleep(0.05)
    assert out == [] and hc.pending == 3
    assert not hc.drain(0.05)
    evs[1].fired.set()
    time.sleep(0.05)
    assert out == []  # FIFO: 1 waits behind 0
    evs[0].fired.set()
    evs[2].fired.set()
    assert hc.drain(5)
    assert out == [0, 1, 2] and hc.pending == 0
    hc.close()


def test_failing_callback_does_not_stop_later_ones():
    hc = HostCompletions("t2")
    out = []
    hc.submit(None, lambda: 1 / 0)
    hc.submit(None, lambda: out.append("ok"))
    assert hc.drain(5) and out == ["ok"]
    hc.close()
