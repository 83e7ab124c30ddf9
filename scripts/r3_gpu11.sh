#!/bin/bash
# GPU suite on this tree, then the ping-pong GEMM: numerics, then TF/s.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export P2PFL_LOCKCHECK=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_pytest_gpu.log 2>&1
rc=$?
tail -4 gpurun_out/r3_pytest_gpu.log
echo "== gemm_pp check"
timeout -k 10 120 python -u scripts/gemm_pp_bench.py --check-only > gpurun_out/gemm_pp_check.log 2>&1 || { cat gpurun_out/gemm_pp_check.log | tail -30; exit 1; }
tail -3 gpurun_out/gemm_pp_check.log
echo "== gemm_pp bench"
timeout -k 10 300 python -u scripts/gemm_pp_bench.py > gpurun_out/gemm_pp_bench.log 2>&1 || { tail -30 gpurun_out/gemm_pp_bench.log; exit 1; }
grep "^|" gpurun_out/gemm_pp_bench.log
exit $rc
