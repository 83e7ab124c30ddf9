#!/bin/bash
# round-3 end-of-session check on this tree: GPU suite, smoke(), N=1 headline bench, configs 3-5 rounds
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export P2PFL_LOCKCHECK=0
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r3_end_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r3_end_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r3_end_pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_end_smoke.log 2>&1 || { tail -20 gpurun_out/r3_end_smoke.log; exit 1; }
tail -1 gpurun_out/r3_end_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r3_end_bench_default.log 2>&1 || { tail -30 gpurun_out/r3_end_bench_default.log; exit 1; }
tail -1 gpurun_out/r3_end_bench_default.log | cut -c1-240
for m in resnet18 resnet50 vit_b16; do
  timeout -k 10 300 python bench.py --model $m --steps 3 --warmup 1 > gpurun_out/r3_end_bench_$m.log 2>&1 || { tail -30 gpurun_out/r3_end_bench_$m.log; exit 1; }
  echo "$m $(tail -1 gpurun_out/r3_end_bench_$m.log | cut -c1-200)"
done
