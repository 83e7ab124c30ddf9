"""Worker for tests/test_xgmi.py: one Node per process on the xGMI transport (gloo data plane on CPU).

    RANK=r WORLD_SIZE=3 MASTER_PORT=p python tests/xgmi_worker.py OUT_JSON fault

``fault``: rank 2 dies (``os._exit(17)``) when the first acknowledgement of
its round-1 model push arrives -- the receiver has accepted the transfer and
launched a receive that can never complete, so the survivors must abort the
communicator and rebuild it over ranks {0, 1}.  Ranks 0 and 1 must still
finish every round with the same model; rank 0 writes the outcome to OUT_JSON.

``twice``: two consecutive experiments on the same nodes; the second must
finish promptly with equal models (no model declined as "already received").

``P2PFL_WORKER_DEVICE=cuda``: the same scenario on the GPU with the RCCL data
plane (no fallback): every rank is its own RCCL "host" (``NCCL_HOSTID`` set by
the test), so three processes on one MI355X form a real 3-rank communicator;
the survivors ``ncclCommAbort`` it and build generation 1 over RCCL.
"""

from __future__ import annotations

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main(out: str, mode: str) -> None:
    from p2pfl_amd.communication.xgmi import XgmiJob
    from p2pfl_amd.data import MnistFederatedDM
    from p2pfl_amd.models import MLP
    from p2pfl_amd.node import Node
    from p2pfl_amd.settings import Settings
    from p2pfl_amd.utils import set_test_settings

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    store = dist.TCPStore("127.0.0.1", int(os.environ["MASTER_PORT"]), world, rank == 0, wait_for_workers=False)
    set_test_settings()
    Settings.LOG_LEVEL = "INFO"
    Settings.TRAIN_SET_SIZE = world
    Settings.GOSSIP_MODELS_PER_ROUND = world - 1
    rounds = 3
    on_gpu = os.environ.get("P2PFL_WORKER_DEVICE", "cpu") == "cuda"
    dev = torch.device("cuda", 0) if on_gpu else torch.device("cpu")
    extra = {}
    if on_gpu:
        from p2pfl_amd import ops

        ops.ext()
        extra = dict(allow_fallback=False)
    job = XgmiJob(rank, world, store, device=dev, backend="rccl" if on_gpu else "gloo", prefix="fault",
                  job_id=f"f{os.environ['MASTER_PORT']}", ack_timeout=3.0, group_timeout=20.0, rebuild_grace=0.5, **extra)
    node = Node(MLP(seed=0), MnistFederatedDM(sub_id=rank, number_sub=4 * world), protocol=job.protocol,
                **({"device": dev} if on_gpu else {}))
    proto = node._communication_protocol
    if mode == "fault" and rank == world - 1:
        orig_start = proto.start

        def start_and_arm():
            orig_start()
            plane = proto.plane
            orig_ack = plane.on_ack

            def dying_ack(seq, epoch, gen):
                if node.state.round == 1:
                    time.sleep(0.2)  # the receiver's group is launched and waits for our send
                    os._exit(17)
                return orig_ack(seq, epoch, gen)

            plane.on_ack = dying_ack

        proto.start = start_and_arm
    node.start()
    addrs = {r: store.get(f"fault/addr/{r}").decode() for r in range(world)}
    for r in range(rank):
        assert node.connect(addrs[r])
    t0 = time.time()
    while len(node.get_neighbors(only_direct=True)) < world - 1:
        assert time.time() - t0 < 60, "mesh did not form"
        time.sleep(0.05)
    store.set(f"up/{rank}", "1")
    store.wait([f"up/{r}" for r in range(world)])
    if rank == 0:
        node.set_start_learning(rounds=rounds, epochs=1)
    t0 = time.time()
    while node._learning_thread is None:
        assert time.time() - t0 < 60
        time.sleep(0.01)
    rounds_done = {"n": 0}
    assert node.wait_learning(timeout=240), "learning did not finish"
    if mode == "twice":
        # a second experiment on the same nodes: it restarts at round 0, so the
        # transport's dedupe keys of the first one must not decline its models
        store.set(f"first/{rank}", "1")
        store.wait([f"first/{r}" for r in range(world)])
        node._learning_thread = None
        if rank == 0:
            node.set_start_learning(rounds=rounds, epochs=1)
        t0 = time.time()
        while node._learning_thread is None:
            assert time.time() - t0 < 60, "second experiment did not start"
            time.sleep(0.01)
        t0 = time.time()
        assert node.wait_learning(timeout=240), "second experiment did not finish"
        assert time.time() - t0 < 60, "second experiment stalled (waited for a timeout)"
    flat = node.state.learner.get_parameters().flat if node.state.learner is not None else None
    s = float(flat.double().sum()) if flat is not None else float("nan")
    digest = ""
    if flat is not None:
        import hashlib

        digest = hashlib.sha1(flat.detach().float().cpu().numpy().tobytes()).hexdigest()
    store.set(f"sum/{rank}", str(s))
    store.set(f"digest/{rank}", digest)
    if rank == 0:
        other = float(store.get("sum/1").decode())
        with open(out, "w") as f:
            json.dump({"rounds": rounds, "rounds_done": rounds if node.state.round is None else node.state.round,
                       "sums": [s, other], "digests": [digest, store.get("digest/1").decode()],
                       "backend": getattr(job, "backend_in_use", None),
                       "stats": dict(proto.plane.stats) if proto.plane else {}}, f)
    store.set(f"done/{rank}", "1")
    store.wait([f"done/{r}" for r in range(world - 1)])
    del rounds_done
    node.stop()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
