"""Lock-order checker (race detection for the control plane)."""

from __future__ import annotations

import threading

import pytest

from p2pfl_amd.utils import lockcheck
from p2pfl_amd.utils.lockcheck import TrackedLock, TrackedRLock


def _new_violations(before):
    return lockcheck.violations()[before:]


@pytest.fixture
def checking():
    was = lockcheck.is_enabled()
    lockcheck.enable(hold_warn_s=10.0)
    yield
    if not was:
        lockcheck.disable()


@pytest.mark.lockcheck_expected
def test_ab_ba_order_is_reported_without_deadlocking(checking):
    a, b = TrackedLock("T1.a"), TrackedLock("T1.b")
    before = len(lockcheck.violations())

    def ab():
        with a:
            with b:
                pass

    def ba():
        with b:
            with a:
                pass

    for fn in (ab, ba):  # sequential: the bad interleaving never happens
        t = threading.Thread(target=fn)
        t.start()
        t.join()
    new = _new_violations(before)
    assert len(new) == 1 and new[0].kind == "class-cycle"
    assert set(new[0].cycle) == {"T1.a", "T1.b"}
    assert "T1.a -> T1.b" in str(new[0])  # the first witness of the other order


def test_consistent_order_and_reentrancy_are_clean(checking):
    a, b, r = TrackedLock("T2.a"), TrackedLock("T2.b"), TrackedRLock("T2.r")
    before = len(lockcheck.violations())
    for _ in range(3):
        with a, b:
            with r:
                with r:  # re-entrant: no self edge
                    pass
    assert _new_violations(before) == []
    rep = lockcheck.report()
    assert "T2.a -> T2.b" in rep["class_edges"] and "T2.b -> T2.r" in rep["class_edges"]


@pytest.mark.lockcheck_expected
def test_same_class_instance_cycle(checking):
    """Two peers' locks of one class taken in both orders (peer1->peer2, peer2->peer1)."""
    p1, p2 = TrackedRLock("T3.peer"), TrackedRLock("T3.peer")
    before = len(lockcheck.violations())
    with p1:
        with p2:
            pass
    with p2:
        with p1:
            pass
    new = _new_violations(before)
    assert [v.kind for v in new] == ["instance-cycle"]


def test_condition_over_tracked_locks(checking):
    for lk in (TrackedLock("T4.l"), TrackedRLock("T4.r")):
        cv = threading.Condition(lk)
        box = []

        def waiter():
            with cv:
                cv.wait_for(lambda: box, timeout=5)
                box.append("seen")

        t = threading.Thread(target=waiter)
        t.start()
        with cv:
            box.append(1)
            cv.notify_all()
        t.join(5)
        assert box == [1, "seen"]
        assert not lk.locked()


def test_semaphore_style_release_from_other_thread(checking):
    """The reference releases locks from other threads (node_state.py:81); no stale state."""
    sem, other = TrackedLock("T5.sem"), TrackedLock("T5.other")
    before = len(lockcheck.violations())
    sem.acquire()
    t = threading.Thread(target=sem.release)
    t.start()
    t.join()
    with other:  # would record T5.sem -> T5.other if the stale entry survived
        pass
    assert "T5.sem -> T5.other" not in lockcheck.report()["class_edges"]
    assert _new_violations(before) == []


@pytest.mark.lockcheck_expected
def test_long_hold_reported(checking):
    lockcheck.enable(hold_warn_s=0.05)
    try:
        lk = TrackedLock("T6.slow")
        before = len(lockcheck.violations())
        with lk:
            threading.Event().wait(0.1)
        new = _new_violations(before)
        assert [v.kind for v in new] == ["long-hold"]
    finally:
        lockcheck.enable(hold_warn_s=10.0)


def test_nodes_run_under_the_checker(protocol):
    """A 2-node learning experiment records the control-plane lock graph, violation-free."""
    if not lockcheck.is_enabled():
        pytest.skip("P2PFL_LOCKCHECK=0")
    from p2pfl_amd.data import MnistFederatedDM
    from p2pfl_amd.models import MLP
    from p2pfl_amd.node import Node
    from p2pfl_amd.utils import check_equal_models, wait_4_results, wait_convergence

    before = len(lockcheck.violations())
    nodes = [Node(MLP(), MnistFederatedDM(sub_id=i, number_sub=2), protocol=protocol) for i in range(2)]
    for n in nodes:
        n.start()
    try:
        nodes[0].connect(nodes[1].addr)
        wait_convergence(nodes, 1, only_direct=True)
        nodes[0].set_start_learning(rounds=2, epochs=0)
        wait_4_results(nodes, timeout=120)
        check_equal_models(nodes)
    finally:
        for n in nodes:
            n.stop()
    assert _new_violations(before) == []
    edges = lockcheck.report()["class_edges"]
    assert edges, "no nested acquisitions were observed"
