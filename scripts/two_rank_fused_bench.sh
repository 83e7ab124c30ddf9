#!/usr/bin/env bash
# Rehearse bench.py's N>1 path on a 1-GPU box: two ranks share the GPU, so the
# collective backend is gloo (RCCL rejects two ranks on one device); the fused
# learner, the FedAvg all-reduce and the JSON contract are exercised as on 8 GPUs.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
P2PFL_DIST_BACKEND=gloo python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 3 --warmup 1
