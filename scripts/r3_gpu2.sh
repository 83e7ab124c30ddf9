#!/bin/bash
# Round-3 GPU check 2: RCCL binding stress (own process), focused GPU tests, N=1 bench, N=2 RCCL rehearsal.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export P2PFL_LOCKCHECK=0
echo "== stress"
timeout -k 10 120 python -u tests/rccl_stress_worker.py 400 > gpurun_out/r3_stress.log 2>&1; rc=$?
cat gpurun_out/r3_stress.log | tail -40
[ $rc -eq 0 ] || exit $rc
echo "== focused tests"
timeout -k 10 900 python -u -m pytest tests/test_gpu_xgmi.py tests/test_gpu_kernels.py tests/test_gpu_cnn_ops.py tests/test_gpu_fused_cnn.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r3_pytest_focus.log 2>&1; rc=$?
tail -15 gpurun_out/r3_pytest_focus.log
[ $rc -eq 0 ] || exit $rc
echo "== bench n1"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r3_bench_n1.log 2>&1 || exit $?
tail -4 gpurun_out/r3_bench_n1.log
echo "== bench n2 rehearsal"
P2PFL_RCCL_SPLIT_HOSTS=1 P2PFL_BENCH_SPANS=1 timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 3 > gpurun_out/r3_bench_n2_rehearsal.log 2>&1 || exit $?
tail -8 gpurun_out/r3_bench_n2_rehearsal.log
