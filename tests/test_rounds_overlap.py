"""Round runner: FedAvg collective overlapped with validation == serial order (gloo, 2 ranks, CPU)."""

from __future__ import annotations

import os
import tempfile

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _worker(rank: int, world: int, init_file: str, out_dir: str) -> None:
    os.environ["P2PFL_LOCKCHECK"] = "0"
    torch.set_num_threads(1)
    dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank, world_size=world)
    try:
        from p2pfl_amd.data import MnistFederatedDM
        from p2pfl_amd.learning.torch_learner import TorchLearner
        from p2pfl_amd.models import MLP
        from p2pfl_amd.parallel.collective import CollectiveFedAvg, DistEnv
        from p2pfl_amd.parallel.rounds import FederatedRoundRunner

        env = DistEnv(rank, world, rank, torch.device("cpu"))
        results = []
        for overlap in (False, True):
            torch.manual_seed(0)
            data = MnistFederatedDM(sub_id=rank, number_sub=40, batch_size=32)
            ln = TorchLearner(MLP(seed=0), data, f"p{rank}", 1, device=torch.device("cpu"))
            runner = FederatedRoundRunner(ln, CollectiveFedAvg(env), overlap_validation=overlap)
            runner.run_round()
            results.append(ln.get_parameters().flat.clone())
        torch.save(results, os.path.join(out_dir, f"r{rank}.pt"))
    finally:
        dist.destroy_process_group()


def test_overlapped_fedavg_matches_serial():
    world = 2
    with tempfile.TemporaryDirectory() as d:
        init = os.path.join(d, "init")
        mp.spawn(_worker, args=(world, init, d), nprocs=world, join=True)
        res = [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True) for r in range(world)]
    for serial, overlapped in res:
        assert torch.equal(serial, overlapped)
    # every peer holds the same aggregate
    assert torch.equal(res[0][1], res[1][1])
    assert not torch.equal(res[0][0], torch.zeros_like(res[0][0]))
