#!/bin/bash
# NaN hunt, step 2: which fresh allocation does fit 2 read before writing?
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export P2PFL_LOCKCHECK=0
run() { echo "== $*"; timeout -k 10 200 python -u scripts/graph_poison.py --fits 2 "$@" > gpurun_out/poison.log 2>&1; rc=$?; grep -E "^fit|held|poisoned|all fits|non-finite|Error|   " gpurun_out/poison.log | head -8; [ $rc -le 2 ] || exit $rc; }
run --hold-only --model resnet50
P2PFL_STEP_GRAPHS=0 run --hold-only --model resnet50
run --fresh nan --model resnet50
run --fresh zero --model resnet50
run --fresh one --model resnet50
run --hold-only --model resnet18
exit 0
