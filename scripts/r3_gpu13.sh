#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export P2PFL_LOCKCHECK=0
echo "== gemm_pp check"
timeout -k 10 120 python -u scripts/gemm_pp_bench.py --check-only > gpurun_out/gemm_pp_check.log 2>&1 || { grep -v amdgpu.ids gpurun_out/gemm_pp_check.log | tail -30; exit 1; }
grep -c OK gpurun_out/gemm_pp_check.log; tail -1 gpurun_out/gemm_pp_check.log
echo "== gemm_pp bench"
timeout -k 10 300 python -u scripts/gemm_pp_bench.py > gpurun_out/gemm_pp_bench.log 2>&1 || { tail -30 gpurun_out/gemm_pp_bench.log; exit 1; }
grep "^|" gpurun_out/gemm_pp_bench.log
bash scripts/r3_gpu12.sh
