#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export P2PFL_LOCKCHECK=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_gemm.py tests/test_gpu_graph_memory.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3_conv_tests.log 2>&1 || { tail -40 gpurun_out/r3_conv_tests.log; exit 1; }
tail -1 gpurun_out/r3_conv_tests.log
timeout -k 10 200 python -u scripts/conv_probe2.py > gpurun_out/conv_probe2.log 2>&1 || { tail -20 gpurun_out/conv_probe2.log; exit 1; }
grep "^|" gpurun_out/conv_probe2.log
timeout -k 10 200 python -u scripts/conv_bench.py --variants 2,2,2 > gpurun_out/conv_bench_find.log 2>&1 || { tail -20 gpurun_out/conv_bench_find.log; exit 1; }
grep -E "^\||ResNet-18 block" gpurun_out/conv_bench_find.log | grep -v "^|---"
timeout -k 10 300 python bench.py --model resnet18 --steps 3 --warmup 1 > gpurun_out/r3_bench_resnet18.log 2>&1 || { tail -30 gpurun_out/r3_bench_resnet18.log; exit 1; }
tail -1 gpurun_out/r3_bench_resnet18.log | cut -c1-220
