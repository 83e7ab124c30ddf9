#!/bin/bash
# Two RCCL ranks on the box's single GPU (distinct NCCL_HOSTID per rank), the
# data plane's epoch-grouped pushes in both directions (tests/rccl_worker.py).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/rccl2
PORT=$((20000 + RANDOM % 20000))
export PYTHONPATH=$PWD P2PFL_LOCKCHECK=0 NCCL_SOCKET_IFNAME=lo NCCL_IB_DISABLE=1 NCCL_DEBUG=${NCCL_DEBUG:-INFO} P2PFL_WORKER_WATCHDOG=80
for r in 0 1; do
  RANK=$r WORLD_SIZE=2 MASTER_PORT=$PORT NCCL_HOSTID=p2pfl-r$r timeout -k 5 100 python -u tests/rccl_worker.py gpurun_out/rccl2/out > gpurun_out/rccl2/rank$r.log 2>&1 &
  pids[$r]=$!
done
rc=0
for r in 0 1; do wait ${pids[$r]} || rc=$?; done
for r in 0 1; do echo "== rank $r"; grep -E "rccl_worker|Error|error|WARN" gpurun_out/rccl2/rank$r.log | tail -25; done
exit $rc
