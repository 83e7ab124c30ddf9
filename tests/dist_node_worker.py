"""Worker for tests/test_dist_protocol.py: one federated Node per process on the xGMI transport.

Run as ``python -m torch.distributed.run --nproc-per-node N tests/dist_node_worker.py OUT_JSON [mlp|cnn]``.
Each rank builds a Node on :class:`~p2pfl_amd.communication.xgmi.XgmiCommunicationProtocol`
(node-local control bus + point-to-point data plane: RCCL with one GPU per
rank, gloo otherwise -- ``P2PFL_XGMI_BACKEND`` overrides), ranks > 0 connect to
rank 0, rank 0 starts a 2-round experiment, and every rank reports its final
parameters' checksum and its data-plane byte counters.
"""

from __future__ import annotations

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main(out: str, model_name: str = "mlp", rounds: int = 2) -> None:
    import faulthandler

    # a hung worker dumps every thread's stack and exits instead of stalling its test
    faulthandler.dump_traceback_later(float(os.environ.get("P2PFL_WORKER_WATCHDOG", "240")), exit=True)
    from p2pfl_amd.communication.xgmi import XgmiJob
    from p2pfl_amd.data import MnistFederatedDM
    from p2pfl_amd.learning.fused_cnn import auto_learner
    from p2pfl_amd.management.logger import logger
    from p2pfl_amd.models import CNN, MLP
    from p2pfl_amd.node import Node
    from p2pfl_amd.settings import Settings
    from p2pfl_amd.utils import set_test_settings

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    dev = torch.device("cuda", local % torch.cuda.device_count()) if torch.cuda.is_available() else torch.device("cpu")
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    dist.init_process_group("gloo")
    store = dist.distributed_c10d._get_default_store()
    set_test_settings()
    Settings.LOG_LEVEL = "INFO"
    job = XgmiJob(rank, world, store, device=dev, backend=os.environ.get("P2PFL_XGMI_BACKEND", "auto"))
    model = MLP(seed=rank) if model_name == "mlp" else CNN(seed=rank)
    node = Node(model, MnistFederatedDM(sub_id=rank, number_sub=2 * world), protocol=job.protocol,
                learner=auto_learner, device=dev)
    node.start()
    try:
        addr0 = store.get(f"{job.prefix}/addr/0").decode()
        if rank > 0:
            assert node.connect(addr0)
        t0 = time.time()
        while len(node.get_neighbors(only_direct=False)) < world - 1:
            if time.time() - t0 > 60:
                raise TimeoutError("neighbour discovery timed out")
            time.sleep(0.1)
        dist.barrier()
        if rank == 0:
            node.set_start_learning(rounds=rounds, epochs=1)
        t0 = time.time()
        while node._learning_thread is None:
            if time.time() - t0 > 120:
                raise TimeoutError("learning never started")
            time.sleep(0.05)
        assert node.wait_learning(timeout=600), "learning did not finish"
        flat = node.state.learner.get_parameters().flat.detach().float().cpu()
        rec = {
            "rank": rank,
            "sum": float(flat.double().sum()),
            "abs": float(flat.double().abs().sum()),
            "metrics": node.state.learner.evaluate(),
            "counters": logger.tracer.counters(node.addr),
            "transport": f"xgmi/{job.backend}",
        }
        objs = [None] * world
        dist.all_gather_object(objs, rec)
        if rank == 0:
            with open(out, "w") as f:
                json.dump(objs, f)
        dist.barrier()  # nobody stops while a peer may still push
    finally:
        node.stop()
        dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1], *(sys.argv[2:3] or ["mlp"]))
