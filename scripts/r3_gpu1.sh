#!/bin/bash
# Round-3 GPU check: full GPU suite, N=1 bench, one-GPU multi-rank RCCL rehearsal.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export P2PFL_LOCKCHECK=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r3_pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/r3_pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r3_bench_n1.log 2>&1 || exit $?
tail -3 gpurun_out/r3_bench_n1.log
P2PFL_RCCL_SPLIT_HOSTS=1 P2PFL_BENCH_SPANS=1 timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 3 > gpurun_out/r3_bench_n2_rehearsal.log 2>&1 || exit $?
tail -3 gpurun_out/r3_bench_n2_rehearsal.log
