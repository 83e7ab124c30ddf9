#!/bin/bash
# verdict r2 #4 follow-up: does a replayed step graph still read freed memory
# (the NaN under rocprofv3)?  Poison every free cached block with NaN after
# the capture, fit again; on NaN, bisect to the block and its allocation site.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export P2PFL_LOCKCHECK=0
run() { echo "== $*"; timeout -k 10 200 python -u scripts/graph_poison.py --fits 2 "$@" > gpurun_out/poison.log 2>&1; rc=$?; grep -E "^fit|poisoned|all fits|non-finite|Error|   " gpurun_out/poison.log | head -20; return $rc; }
run --poison --model resnet50
rc=$?
if [ $rc -eq 2 ]; then
  timeout -k 10 400 python -u scripts/graph_uaf_bisect.py --model resnet50 > gpurun_out/uaf_bisect.log 2>&1
  tail -40 gpurun_out/uaf_bisect.log
  exit 0
fi
[ $rc -eq 0 ] || exit $rc
P2PFL_NATIVE_CONV=1 P2PFL_NATIVE_GEMM=1 run --poison --model resnet18 || exit $?
run --poison --model vit_tiny
