#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export P2PFL_LOCKCHECK=0
echo "== rccl 2 ranks on one GPU"
NCCL_DEBUG=WARN timeout -k 10 130 bash scripts/r3_rccl2.sh || exit $?
echo "== focused tests"
timeout -k 10 1000 python -u -m pytest tests/test_gpu_cnn_ops.py tests/test_gpu_fused_cnn.py tests/test_gpu_kernels.py tests/test_gpu_xgmi.py -x -v --timeout 170 --timeout-method thread > gpurun_out/r3_pytest_focus.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r3_pytest_focus.log | tail -12
[ $rc -eq 0 ] || { tail -60 gpurun_out/r3_pytest_focus.log; exit $rc; }
echo "== bench n1"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r3_bench_n1.log 2>&1 || { tail -30 gpurun_out/r3_bench_n1.log; exit 1; }
tail -4 gpurun_out/r3_bench_n1.log
echo "== bench n2 rehearsal"
P2PFL_RCCL_SPLIT_HOSTS=1 P2PFL_BENCH_SPANS=1 timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 3 > gpurun_out/r3_bench_n2_rehearsal.log 2>&1 || { tail -30 gpurun_out/r3_bench_n2_rehearsal.log; exit 1; }
tail -12 gpurun_out/r3_bench_n2_rehearsal.log
