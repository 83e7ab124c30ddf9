#!/bin/bash
# full GPU suite; conv probes; ResNet-18 / ResNet-50 / headline benches
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export P2PFL_LOCKCHECK=0
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r3_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r3_pytest_gpu.log
timeout -k 10 200 python -u scripts/conv_probe2.py > gpurun_out/conv_probe2.log 2>&1 || { tail -20 gpurun_out/conv_probe2.log; exit 1; }
grep "^|" gpurun_out/conv_probe2.log
timeout -k 10 200 python -u scripts/conv_bench.py --variants 2,2,2 > gpurun_out/conv_bench_find.log 2>&1 || { tail -20 gpurun_out/conv_bench_find.log; exit 1; }
grep -E "ResNet-18 block" gpurun_out/conv_bench_find.log
for m in resnet18 resnet50; do
timeout -k 10 300 python bench.py --model $m --steps 3 --warmup 1 > gpurun_out/r3_bench_$m.log 2>&1 || { tail -30 gpurun_out/r3_bench_$m.log; exit 1; }
tail -1 gpurun_out/r3_bench_$m.log | cut -c1-220
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r3_bench_n1.log 2>&1 || { tail -30 gpurun_out/r3_bench_n1.log; exit 1; }
tail -1 gpurun_out/r3_bench_n1.log | cut -c1-250
