#!/bin/bash
cd "$(dirname "$0")/.."
export P2PFL_LOCKCHECK=0
run() { echo "== $*"; timeout -k 10 120 python -u scripts/graph_poison.py --fits 2 "$@" 2>&1 | grep -vE "^W2026|amdgpu.ids" ; }
run --hold-only
run --poison
P2PFL_NATIVE_CONV=0 P2PFL_NATIVE_GEMM=0 run --poison
exit 0
