#!/bin/bash
# GEMM tests after the weight-gradient split cap change + ResNet-50 / ResNet-18 rounds on the new default
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export P2PFL_LOCKCHECK=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_graph_memory.py tests/test_gpu_step_graph.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3_split_pytest.log 2>&1 || { tail -40 gpurun_out/r3_split_pytest.log; exit 1; }
tail -1 gpurun_out/r3_split_pytest.log
for m in resnet50 resnet18; do
  timeout -k 10 300 python bench.py --model $m --steps 3 --warmup 1 > gpurun_out/r3_split_default_$m.log 2>&1 || { tail -30 gpurun_out/r3_split_default_$m.log; exit 1; }
  echo "$m $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r3_split_default_$m.log)"
done
