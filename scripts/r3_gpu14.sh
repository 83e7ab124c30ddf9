#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export P2PFL_LOCKCHECK=0
timeout -k 10 200 python -u scripts/gemm_pp_bench.py --probes > gpurun_out/gemm_pp_probes.log 2>&1 || { tail -30 gpurun_out/gemm_pp_probes.log; exit 1; }
grep "^|" gpurun_out/gemm_pp_probes.log
bash scripts/r3_gpu12.sh
