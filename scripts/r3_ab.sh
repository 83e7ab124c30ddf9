#!/bin/bash
# A/B of the fused CNN kernels + a kernel-trace profile of the default path.
set -o pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
cd "$ROOT"; mkdir -p gpurun_out/ab
export P2PFL_LOCKCHECK=0
for v in "1 1" "0 1" "1 0" "0 0"; do
  set -- $v
  P2PFL_CNN_FUSED_CONV=$1 P2PFL_CNN_FUSED_HEAD=$2 P2PFL_BENCH_SPANS=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/ab/conv$1_head$2.log 2>&1 || exit $?
  echo "conv=$1 head=$2: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab/conv$1_head$2.log)"
  grep "all spans" gpurun_out/ab/conv$1_head$2.log | cut -c1-400
done
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/ab/prof" -o run -- python3 "$ROOT/bench.py" --steps 20 --warmup 5 > "$ROOT/gpurun_out/ab/prof.log" 2>&1 || exit $?
find "$ROOT/gpurun_out/ab/prof" -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'head -16 {}'
