#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export P2PFL_LOCKCHECK=0
timeout -k 10 200 python -u scripts/conv_probe2.py > gpurun_out/conv_probe2.log 2>&1 || { tail -20 gpurun_out/conv_probe2.log; exit 1; }
grep "^|" gpurun_out/conv_probe2.log
timeout -k 10 200 python -u scripts/conv_bench.py --variants 2,2,2 > gpurun_out/conv_bench_find.log 2>&1 || { tail -20 gpurun_out/conv_bench_find.log; exit 1; }
grep -E "^\||ResNet-18 block" gpurun_out/conv_bench_find.log | grep -v "^|---"
