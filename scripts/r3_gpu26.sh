#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export P2PFL_LOCKCHECK=0
timeout -k 10 200 python -u scripts/conv_probe2.py > gpurun_out/conv_probe2.log 2>&1 || { tail -20 gpurun_out/conv_probe2.log; exit 1; }
grep "^|" gpurun_out/conv_probe2.log
