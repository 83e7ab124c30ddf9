#!/bin/bash
# NaN hunt, step 3: which path needs the freed memory (library GEMMs / TunableOp, native convs), and which step turns non-finite
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export P2PFL_LOCKCHECK=0
run() { echo "== $*"; timeout -k 10 200 python -u scripts/graph_poison.py --fits 2 "$@" > gpurun_out/poison.log 2>&1; rc=$?; grep -E "^fit|all fits|   replay|   after|Error" gpurun_out/poison.log | head -8; [ $rc -le 2 ] || exit $rc; }
run --hold-only --model resnet50 --trace-steps
P2PFL_TUNABLEOP=0 run --hold-only --model resnet50
P2PFL_NATIVE_CONV=0 P2PFL_NATIVE_GEMM=0 run --hold-only --model resnet50
P2PFL_NATIVE_CONV=1 run --hold-only --model resnet50
exit 0
