#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export P2PFL_LOCKCHECK=0
echo "== bench n1"
P2PFL_BENCH_SPANS=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/r3_bench_n1.log 2>&1 || { tail -30 gpurun_out/r3_bench_n1.log; exit 1; }
grep -E "all spans|ms_per_step" gpurun_out/r3_bench_n1.log | cut -c1-600
echo "== nan hunt (profiled, overlap off)"
bash scripts/r3_nan_hunt.sh off
