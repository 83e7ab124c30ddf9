#!/bin/bash
# NaN hunt, step 4: MIOpen GEMM-based solvers off (old routing), then the 1x1-as-GEMM routing
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export P2PFL_LOCKCHECK=0
run() { echo "== $*"; timeout -k 10 200 python -u scripts/graph_poison.py --fits 2 "$@" > gpurun_out/poison.log 2>&1; rc=$?; grep -E "^fit|all fits|   replay|Error" gpurun_out/poison.log | head -6; [ $rc -le 2 ] || exit $rc; }
P2PFL_CONV1X1_GEMM=0 MIOPEN_DEBUG_CONV_GEMM=0 run --hold-only --model resnet50
run --hold-only --model resnet50
run --poison --model resnet50
run --fresh nan --model resnet50
exit 0
