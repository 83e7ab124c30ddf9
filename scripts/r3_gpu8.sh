#!/bin/bash
cd "$(dirname "$0")/.."
export P2PFL_LOCKCHECK=0
run() { echo "== $*"; timeout -k 10 150 python -u scripts/graph_poison.py --poison --fits 2 "$@" 2>&1 | grep -E "^fit|poisoned|all fits|Error" ; }
run --model mlp
run --model vit_tiny
P2PFL_NATIVE_CONV=1 P2PFL_NATIVE_GEMM=1 run --model resnet18
P2PFL_NATIVE_CONV=0 P2PFL_NATIVE_GEMM=0 run --model resnet18
exit 0
