#!/bin/bash
# weight-gradient split-K cap of ops.gemm (1x1-conv GEMMs of ResNet-50): A/B over the round time
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export P2PFL_LOCKCHECK=0
for cap in 16 64 16 64; do
  P2PFL_GEMM_MAX_SPLITS=$cap timeout -k 10 300 python bench.py --model resnet50 --steps 3 --warmup 1 > gpurun_out/r3_split_r50_$cap.log 2>&1 || { tail -30 gpurun_out/r3_split_r50_$cap.log; exit 1; }
  echo "cap=$cap $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r3_split_r50_$cap.log)"
done
for cap in 16 64; do
  P2PFL_GEMM_MAX_SPLITS=$cap timeout -k 10 300 python bench.py --model resnet18 --steps 3 --warmup 1 > gpurun_out/r3_split_r18_$cap.log 2>&1 || { tail -30 gpurun_out/r3_split_r18_$cap.log; exit 1; }
  echo "r18 cap=$cap $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r3_split_r18_$cap.log)"
done
