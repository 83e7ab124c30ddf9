#!/bin/bash
# full GPU suite on this tree; N=1 headline bench; the 8-peer ResNet-50 scenario under
# rocprofv3 (NaN fix check); ViT-B/16 and ResNet-18 rounds with the autotune decisions
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export P2PFL_LOCKCHECK=0
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r3_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r3_pytest_gpu.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r3_bench_n1.log 2>&1 || { tail -30 gpurun_out/r3_bench_n1.log; exit 1; }
tail -1 gpurun_out/r3_bench_n1.log
bash scripts/r3_nan_hunt.sh fix --rounds 6 || exit $?
timeout -k 10 300 python bench.py --model resnet18 --steps 3 --warmup 1 > gpurun_out/r3_bench_resnet18.log 2>&1 || { tail -30 gpurun_out/r3_bench_resnet18.log; exit 1; }
tail -1 gpurun_out/r3_bench_resnet18.log
timeout -k 10 400 python bench.py --model vit_b16 --steps 2 --warmup 1 > gpurun_out/r3_bench_vit.log 2>&1 || { tail -30 gpurun_out/r3_bench_vit.log; exit 1; }
tail -1 gpurun_out/r3_bench_vit.log
