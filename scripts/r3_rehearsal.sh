#!/bin/bash
# One-GPU rehearsal of the multi-rank bench at N = 2, 4, 8: every rank is its
# own RCCL "host" (distinct NCCL_HOSTID, RCCL socket transport on loopback),
# all ranks time-share the single GPU.  Checks the N-rank protocol + RCCL path
# end to end; the timings are NOT xGMI scaling numbers.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/rehearsal
export P2PFL_LOCKCHECK=0 P2PFL_RCCL_SPLIT_HOSTS=1 P2PFL_BENCH_SPANS=1
for n in ${@:-2 4 8}; do
  echo "== N=$n"
  timeout -k 10 240 python bench.py --gpus $n --steps 6 --warmup 2 --watchdog 200 > gpurun_out/rehearsal/n$n.log 2>&1
  rc=$?
  grep -E '^\{' gpurun_out/rehearsal/n$n.log | python3 -c "import sys,json; [print({k: d[k] for k in ('n_gpus','ms_per_step','value','transport')}) for d in map(json.loads, sys.stdin)]"
  grep -E "per-round \(mean" gpurun_out/rehearsal/n$n.log | head -8
  [ $rc -eq 0 ] || { echo "N=$n failed rc=$rc"; tail -20 gpurun_out/rehearsal/n$n.log; exit $rc; }
done
