#!/bin/bash
# round-3 final check on this tree: GPU suite, smoke(), N=1 headline bench, 2-rank RCCL rehearsal
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export P2PFL_LOCKCHECK=0
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r3_final_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r3_final_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r3_final_pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_final_smoke.log 2>&1 || { tail -20 gpurun_out/r3_final_smoke.log; exit 1; }
tail -1 gpurun_out/r3_final_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r3_final_bench_default.log 2>&1 || { tail -30 gpurun_out/r3_final_bench_default.log; exit 1; }
tail -1 gpurun_out/r3_final_bench_default.log | cut -c1-200
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r3_final_bench_n1.log 2>&1 || { tail -30 gpurun_out/r3_final_bench_n1.log; exit 1; }
tail -1 gpurun_out/r3_final_bench_n1.log | cut -c1-200
timeout -k 10 300 python bench.py --model resnet18 --steps 3 --warmup 1 > gpurun_out/r3_final_bench_resnet18.log 2>&1 || { tail -30 gpurun_out/r3_final_bench_resnet18.log; exit 1; }
tail -1 gpurun_out/r3_final_bench_resnet18.log | cut -c1-200
P2PFL_RCCL_SPLIT_HOSTS=1 P2PFL_BENCH_SPANS=1 timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 3 > gpurun_out/r3_final_bench_n2_rehearsal.log 2>&1 || { tail -30 gpurun_out/r3_final_bench_n2_rehearsal.log; exit 1; }
grep '"metric"' gpurun_out/r3_final_bench_n2_rehearsal.log | cut -c1-200
timeout -k 10 200 python -u scripts/wgrad_splits_probe.py > gpurun_out/wgrad_splits_probe.log 2>&1 || { tail -20 gpurun_out/wgrad_splits_probe.log; exit 1; }
grep "^|" gpurun_out/wgrad_splits_probe.log
