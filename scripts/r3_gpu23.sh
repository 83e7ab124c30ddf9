#!/bin/bash
# native conv: 4-stage ring (variant bit 12) vs the round-2 schedules, ResNet-18 CIFAR shapes, batch 32
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export P2PFL_LOCKCHECK=0
timeout -k 10 200 python -u -m pytest tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3_conv_tests.log 2>&1 || { tail -30 gpurun_out/r3_conv_tests.log; exit 1; }
tail -1 gpurun_out/r3_conv_tests.log
for v in 10,10,2 4098,4098,4098 2,2,2; do
  echo "== variants $v"
  timeout -k 10 200 python -u scripts/conv_bench.py --variants $v > gpurun_out/conv_bench_$v.log 2>&1 || { tail -20 gpurun_out/conv_bench_$v.log; exit 1; }
  grep -E "^\||ResNet-18 block" gpurun_out/conv_bench_$v.log
done
