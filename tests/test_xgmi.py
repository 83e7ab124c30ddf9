"""xGMI transport: epoch-ordered data plane, control bus, multi-process runs, peer failure.

* the strict RCCL simulator really deadlocks on the naive schedule (so passing
  against it means something);
* concurrent random pushes between several ranks through the epoch scheduler
  always complete with intact payloads (deadlock freedom, property test);
* k peers pushing to each other simultaneously over real processes (gloo
  backend) -- the full Node stack, via ``bench.py --gpus 3`` with no launcher;
* a rank killed in the middle of a transfer: the survivors finish every round.
"""

from __future__ import annotations

import json
import os
import random
import socket
import subprocess
import sys
import threading
import time

import pytest
import torch

from p2pfl_amd.communication.xgmi.bus import BusEndpoint
from p2pfl_amd.communication.xgmi.data_plane import RECV, SEND, SimFabric, XgmiDataPlane, make_backend_factory

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_sim_fabric_models_rccl_stream_order_deadlock():
    """Two ranks that each launch [send] then [recv] as separate groups deadlock
    on RCCL (each stream blocks on a send whose receive is queued behind the
    peer's own send); the simulator must reproduce that, and the same four
    operations issued as ONE group per rank must complete."""
    f = SimFabric()
    a, b = torch.arange(4.0), torch.arange(4.0) + 10
    ra, rb = torch.empty(4), torch.empty(4)
    g = [f.issue(0, [(SEND, 1, a)]), f.issue(1, [(SEND, 0, b)]), f.issue(0, [(RECV, 1, ra)]), f.issue(1, [(RECV, 0, rb)])]
    time.sleep(0.05)
    assert not any(x.done.is_set() for x in g)
    f2 = SimFabric()
    g2 = [f2.issue(0, [(SEND, 1, a), (RECV, 1, ra)]), f2.issue(1, [(SEND, 0, b), (RECV, 0, rb)])]
    assert all(x.done.wait(1) for x in g2)
    assert torch.equal(ra, b) and torch.equal(rb, a)


class _Mesh:
    """n in-process data planes on one simulated fabric, wired like the transport does it."""

    def __init__(self, n: int) -> None:
        import torch.distributed as dist

        self.fabric = SimFabric()
        self.store = dist.HashStore()
        self.planes = [
            XgmiDataPlane(r, n, make_backend_factory("sim", r, self.store, "t", torch.device("cpu"), self.fabric),
                          store=self.store, prefix="t", ack_timeout=5, group_timeout=10, preconnect=False)
            for r in range(n)
        ]
        for p in self.planes:
            p.start(block=True)
        self.received = {r: [] for r in range(n)}
        self.lock = threading.Lock()

    def push(self, src: int, dst: int, t: torch.Tensor, done: threading.Semaphore) -> None:
        """What the transport does: propose, header to the receiver, accept, ack."""
        def on_send(ok, reason, evict):
            assert ok, reason
            done.release()

        hdr = self.planes[src].propose(dst, t, on_send)

        def on_recv(buf, reason):
            assert buf is not None, reason
            with self.lock:
                self.received[dst].append((src, buf.clone()))
            done.release()

        # header / ack travel on other threads, at arbitrary moments
        def receiver():
            time.sleep(random.random() * 0.002)
            e, why = self.planes[dst].accept(src, hdr, on_recv)
            assert e is not None, why
            time.sleep(random.random() * 0.002)
            self.planes[src].on_ack(hdr["seq"], e, hdr["gen"])

        threading.Thread(target=receiver, daemon=True).start()

    def stop(self) -> None:
        for p in self.planes:
            p.stop()


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_epoch_plane_random_concurrent_pushes_never_deadlock(seed):
    rng = random.Random(seed)
    random.seed(seed)
    n = 5
    mesh = _Mesh(n)
    try:
        done = threading.Semaphore(0)
        expected = 0
        sent = {r: [] for r in range(n)}

        def sender(src):
            for _ in range(12):
                k = rng.randint(1, n - 1)
                for dst in rng.sample([r for r in range(n) if r != src], k):
                    t = torch.full((257,), float(src * 1000 + len(sent[src])))
                    sent[src].append((dst, t))
                    mesh.push(src, dst, t, done)
                time.sleep(rng.random() * 0.003)

        threads = [threading.Thread(target=sender, args=(r,)) for r in range(n)]
        for th in threads:
            th.start()
        for th in threads:
            th.join()
        expected = 2 * sum(len(v) for v in sent.values())
        for _ in range(expected):
            assert done.acquire(timeout=20), "transfers stalled (deadlock)"
        # every payload arrived intact at its destination
        for src, lst in sent.items():
            for dst, t in lst:
                assert any(s == src and torch.equal(b, t) for s, b in mesh.received[dst])
        assert sum(p.stats["groups"] for p in mesh.planes) > 0
    finally:
        mesh.stop()


def test_bus_detects_dead_peer_and_keeps_order():
    got, closed = [], []
    a = BusEndpoint("busA-test", lambda src, data: got.append((src, data)), lambda src: closed.append(src))
    b = BusEndpoint("busB-test", lambda src, data: None)
    a.start()
    b.start()
    try:
        for i in range(200):
            b.send("busA-test", str(i).encode())
        t0 = time.time()
        while len(got) < 200 and time.time() - t0 < 5:
            time.sleep(0.01)
        assert [int(d) for _, d in got] == list(range(200)) and all(s == "busB-test" for s, _ in got)
        b.close()
        t0 = time.time()
        while not closed and time.time() - t0 < 5:
            time.sleep(0.01)
        assert closed == ["busB-test"]
        with pytest.raises(ConnectionError):
            BusEndpoint("busC-test", lambda *a: None).send("no-such-node", b"x")
    finally:
        a.close()
        b.close()


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _env():
    return dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1",
                P2PFL_LOCKCHECK="0")


@pytest.mark.timeout(600)
def test_three_processes_push_to_each_other_full_stack():
    """bench.py launches 3 worker processes itself (no torchrun); every round each
    peer pushes its model to both others at the same moment (fan-out 2)."""
    cmd = [sys.executable, "bench.py", "--gpus", "3", "--steps", "2", "--warmup", "1", "--impl", "torch",
           "--number-sub", "400", "--watchdog", "240"]
    r = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=560)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    rec = lines[0]
    assert rec["n_gpus"] == 3 and rec["config"]["parallelism"] == "gossip-p2p"
    assert rec["transport"] == "xgmi/gloo"
    # each rank's per-round line: it received the two other models every round
    recvs = [ln for ln in r.stderr.splitlines() if "data plane:" in ln]
    assert len(recvs) == 3


def _plane_lines(stderr: str):
    """rank -> (sends, receives, MB sent) from bench.py's per-rank summary lines."""
    import re

    out = {}
    for ln in stderr.splitlines():
        m = re.search(r"\[bench rank (\d+)\] per-round .*data plane: (\d+) sends / (\d+) recvs .*xgmi bytes sent ([\d.]+) MB", ln)
        if m:
            out[int(m.group(1))] = (int(m.group(2)), int(m.group(3)), float(m.group(4)))
    return out


@pytest.mark.timeout(600)
@pytest.mark.parametrize("n", [4, 6])
def test_full_mesh_round_moves_each_model_exactly_once(n):
    """Full mesh, every peer in the train set: each round every model crosses
    each link once -- N - 1 pushes per rank per round, plus the N - 1 pushes of
    the initial model -- and nothing else (no relayed partials, no diffusion of
    the full aggregate to peers that finish on their own).  Reference schedule
    being replaced: gossip_model_stage.py:100-104, gossiper.py:228-239."""
    W, K = 1, 2
    cmd = [sys.executable, "bench.py", "--gpus", str(n), "--steps", str(K), "--warmup", str(W), "--impl", "torch",
           "--number-sub", "800", "--watchdog", "300"]
    r = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=560)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = _plane_lines(r.stderr)
    assert sorted(lines) == list(range(n)), r.stderr[-3000:]
    rounds = W + K
    total_sends = sum(v[0] for v in lines.values())
    assert total_sends == rounds * n * (n - 1) + (n - 1), lines
    assert sum(v[1] for v in lines.values()) == total_sends
    for rank, (sends, _, _) in lines.items():
        assert rounds * (n - 1) <= sends <= (rounds + 1) * (n - 1), (rank, lines)


@pytest.mark.timeout(600)
def test_rank_killed_mid_transfer_survivors_finish():
    port = _free_port()
    out = os.path.join("/tmp", f"xgmi_fault_{port}.json")
    env = _env()
    procs = []
    for r in range(3):
        e = dict(env, RANK=str(r), WORLD_SIZE="3", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "xgmi_worker.py"), out, "fault"],
                                      cwd=ROOT, env=e, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    for p in procs:
        try:
            o, _ = p.communicate(timeout=300)
        except subprocess.TimeoutExpired:
            p.kill()
            o, _ = p.communicate()
        outs.append(o)
    assert procs[2].returncode == 17, outs[2][-3000:]  # the victim died on purpose
    assert procs[0].returncode == 0, outs[0][-4000:]
    assert procs[1].returncode == 0, outs[1][-4000:]
    with open(out) as f:
        rec = json.load(f)
    os.unlink(out)
    assert rec["rounds_done"] == rec["rounds"]
    assert rec["stats"].get("rebuilds", 0) >= 1  # the stuck receive forced a new communicator
    # the survivors ended with the same model
    assert abs(rec["sums"][0] - rec["sums"][1]) < 1e-3 * max(1.0, abs(rec["sums"][0]))


@pytest.mark.timeout(600)
def test_two_consecutive_experiments_on_the_same_nodes():
    """A second experiment restarts at round 0 with the same (round, command,
    contributors) as the first: the transport's dedupe of received models is per
    experiment, so nothing is declined and no node waits for a timeout."""
    port = _free_port()
    out = os.path.join("/tmp", f"xgmi_twice_{port}.json")
    env = _env()
    procs = []
    for r in range(3):
        e = dict(env, RANK=str(r), WORLD_SIZE="3", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "xgmi_worker.py"), out, "twice"],
                                      cwd=ROOT, env=e, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    for p in procs:
        try:
            o, _ = p.communicate(timeout=400)
        except subprocess.TimeoutExpired:
            p.kill()
            o, _ = p.communicate()
        outs.append(o)
    for r, p in enumerate(procs):
        assert p.returncode == 0, outs[r][-4000:]
    with open(out) as f:
        rec = json.load(f)
    os.unlink(out)
    assert rec["digests"][0] == rec["digests"][1]


def test_primary_backend_failure_on_one_rank_switches_every_rank_to_fallback():
    import torch.distributed as dist

    from p2pfl_amd.communication.xgmi.data_plane import SimBackend

    fabric, store = SimFabric(), dist.HashStore()

    def primary(rank):
        def make(gen, members):
            if rank == 1:
                raise RuntimeError("no RCCL here")
            return SimBackend(SimFabric(), members, rank)  # a fabric nobody else uses
        return make

    planes = []
    for r in range(2):
        p = XgmiDataPlane(r, 2, primary(r), store=store, prefix="fb", preconnect=False, group_timeout=10)
        p.fallback = make_backend_factory("sim", r, store, "fb", torch.device("cpu"), fabric)
        planes.append(p)
    for p in planes:
        p.start()
    try:
        for p in planes:
            assert p.ready.wait(10) and p.failed is None
            assert p._backend.fabric is fabric  # both on the agreed fallback
        got = threading.Event()
        t = torch.arange(8.0)
        hdr = planes[0].propose(1, t, lambda ok, reason, evict: None)
        e, _ = planes[1].accept(0, hdr, lambda buf, reason: (got.set() if buf is not None and torch.equal(buf, t) else None))
        planes[0].on_ack(hdr["seq"], e, hdr["gen"])
        assert got.wait(10)
    finally:
        for p in planes:
            p.stop()


def test_bus_carries_records_larger_than_one_packet():
    """A record above MAX_RECORD (the fallback path of a model the data plane
    cannot carry) arrives intact, in order with the small records around it,
    and the bulk connection that carried it does not count as the peer leaving."""
    from p2pfl_amd.communication.xgmi.bus import MAX_RECORD

    got, closed = [], []
    a = BusEndpoint("busA-frag", lambda src, data: got.append(data), lambda src: closed.append(src))
    b = BusEndpoint("busB-frag", lambda src, data: None)
    a.start()
    b.start()
    try:
        big = bytes(random.Random(0).getrandbits(8) for _ in range(4096)) * (3 * MAX_RECORD // 4096 + 7)
        b.send("busA-frag", b"before")
        b.send("busA-frag", big)
        b.send("busA-frag", b"after")
        b.send("busA-frag", big[: MAX_RECORD + 1])
        t0 = time.time()
        while len(got) < 4 and time.time() - t0 < 10:
            time.sleep(0.01)
        small = [g for g in got if len(g) < 16]
        large = [g for g in got if len(g) >= 16]
        assert small == [b"before", b"after"]
        assert large == [big, big[: MAX_RECORD + 1]]
        b.drop("busA-frag")  # closes both connections: the main one reports the exit
        t0 = time.time()
        while not closed and time.time() - t0 < 5:
            time.sleep(0.01)
        assert closed == ["busB-frag"]
    finally:
        a.close()
        b.close()


def test_unusable_data_plane_still_delivers_models_larger_than_a_bus_packet():
    """With the data plane down (init/rebuild failed), a 26 MB CNN must still
    reach the peer over the control bus instead of evicting the neighbour."""
    from p2pfl_amd.communication.xgmi import XgmiSimNetwork
    from p2pfl_amd.data import MnistFederatedDM
    from p2pfl_amd.models import CNN
    from p2pfl_amd.node import Node
    from p2pfl_amd.utils import check_equal_models, wait_4_results, wait_convergence

    net = XgmiSimNetwork()
    nodes = [Node(CNN(seed=i), MnistFederatedDM(sub_id=i, number_sub=400), protocol=net.protocol) for i in range(2)]
    for nd in nodes:
        nd.start()
    try:
        nodes[1].connect(nodes[0].addr)
        wait_convergence(nodes, 1, only_direct=True, wait=10)
        for nd in nodes:
            plane = nd._communication_protocol.plane
            assert plane.ready.wait(10)
            plane.failed = "forced off by the test"
        nodes[0].set_start_learning(rounds=1, epochs=0)
        wait_4_results(nodes, timeout=120)
        check_equal_models(nodes)
        # still neighbours: nobody was dropped for an oversized record
        assert nodes[1].addr in nodes[0].get_neighbors(only_direct=True)
    finally:
        for nd in nodes:
            nd.stop()


def test_late_rank_rejoins_next_generation_instead_of_failing():
    """A survivor that announces after the others agreed on generation g
    requests g + 1, and every survivor ends in the same generation."""
    import torch.distributed as dist

    from p2pfl_amd.communication.xgmi.data_plane import agree_members

    store = dist.HashStore()
    # ranks 0 and 1 agree on g1 without rank 2 (it is late: its announcement
    # has not arrived within their wait)
    got = agree_members(store, "lj", 1, 0, 3, [], 0.0, wait_all=0.05)
    assert got == [0]
    assert agree_members(store, "lj", 1, 1, 3, [], 0.0, wait_all=0.05) == [0]
    # rank 2 is excluded from g1: it announces for g2 and then asks for it;
    # g2 includes everyone who announced, even a rank written off as lost
    store.set("lj/g2/alive/2", "1")
    res = {}
    ths = [threading.Thread(target=lambda r=r: res.__setitem__(r, agree_members(store, "lj", 2, r, 3, [2] if r < 2 else [], 0.0, wait_all=2.0)))
           for r in range(3)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert res[0] == res[1] == res[2] == [0, 1, 2]


def test_plane_fallback_disallowed_fails_loudly():
    import torch.distributed as dist

    from p2pfl_amd.communication.xgmi.data_plane import SimBackend

    fabric, store = SimFabric(), dist.HashStore()

    def primary(rank):
        def make(gen, members):
            if rank == 1:
                raise RuntimeError("no RCCL here")
            return SimBackend(fabric, members, rank)
        return make

    planes = []
    for r in range(2):
        p = XgmiDataPlane(r, 2, primary(r), store=store, prefix="nf", preconnect=False, group_timeout=10)
        p.fallback = make_backend_factory("sim", r, store, "nf", torch.device("cpu"), fabric)
        p.allow_fallback = False
        planes.append(p)
    for p in planes:
        p.start()
    try:
        for p in planes:
            assert p.ready.wait(10)
            assert p.failed is not None and "fallback disallowed" in p.failed and "[1]" in p.failed
            assert not p.usable
    finally:
        for p in planes:
            p.stop()


@pytest.mark.timeout(600)
def test_bench_reports_the_backend_actually_used():
    """--plane-backend rccl on a machine without RCCL: with --allow-fallback the
    JSON says xgmi/gloo (the fallback is never reported as rccl); without it the
    run fails instead of producing a mislabelled number."""
    base = [sys.executable, "bench.py", "--gpus", "2", "--steps", "1", "--warmup", "0", "--impl", "torch",
            "--number-sub", "400", "--watchdog", "240", "--plane-backend", "rccl"]
    r = subprocess.run(base + ["--allow-fallback"], cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=560)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    rec = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")][0]
    assert rec["transport"] == "xgmi/gloo"
    # per-rank, per-round breakdown on stderr at N > 1
    assert any("round 1: wall" in ln and "pushes: ack" in ln for ln in r.stderr.splitlines()), r.stderr[-3000:]
    r = subprocess.run(base, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=560)
    assert r.returncode != 0
    assert "fallback disallowed" in (r.stdout + r.stderr)
